// devtest.hip -- device-level unit tests of building blocks (built as libadmm_devtest.so; used only by
// tests/test_gpu_devtest.py, never by the product path).
#include <hip/hip_runtime.h>

#include "layout.hpp"
#include "line_pair.hpp"
#include "line_quad.hpp"
#include "plane_kernel.hip"
#include "capi_internal.hpp"

namespace {

// one block = 512 threads = 256 lines (lane pair per line)
__global__ __launch_bounds__(512) void pair_fwd_kernel(const float* __restrict__ x, float2* __restrict__ spec) {
    const int r = blockIdx.x * 256 + (threadIdx.x >> 1);
    const bool hb = threadIdx.x & 1;
    const float2* row = reinterpret_cast<const float2*>(x + (size_t)r * 256) + (hb ? 1 : 0);
    float2 S[64];
#pragma unroll
    for (int n = 0; n < 64; ++n) S[n] = row[2 * n];
    admm::line_forward_pair(S, hb);
    float2* out = spec + (size_t)r * 128 + (hb ? 64 : 0);
#pragma unroll
    for (int m = 0; m < 64; ++m) out[m] = S[m];
}

__global__ __launch_bounds__(512) void pair_inv_kernel(const float2* __restrict__ spec, float* __restrict__ x) {
    const int r = blockIdx.x * 256 + (threadIdx.x >> 1);
    const bool hb = threadIdx.x & 1;
    const float2* in = spec + (size_t)r * 128 + (hb ? 64 : 0);
    float2 S[64];
#pragma unroll
    for (int m = 0; m < 64; ++m) S[m] = in[m];
    admm::line_inverse_pair(S, hb);
    float2* row = reinterpret_cast<float2*>(x + (size_t)r * 256) + (hb ? 1 : 0);
#pragma unroll
    for (int n = 0; n < 64; ++n) row[2 * n] = S[n];
}

// lane-quad layout: one block = 1024 threads = 256 lines
__global__ __launch_bounds__(1024) void quad_fwd_kernel(const float* __restrict__ x, float2* __restrict__ spec) {
    const int r = blockIdx.x * 256 + (threadIdx.x >> 2);
    const admm::quad::Lane L = admm::quad::lane_of(threadIdx.x);
    const float2* row = reinterpret_cast<const float2*>(x + (size_t)r * 256) + L.q;
    float2 S[32];
#pragma unroll
    for (int m = 0; m < 32; ++m) S[m] = row[4 * m];
    admm::quad::line_forward(S, L);
    float2* out = spec + (size_t)r * 128 + 32 * L.p;
#pragma unroll
    for (int k = 0; k < 32; ++k) out[k] = S[k];
}

__global__ __launch_bounds__(1024) void quad_inv_kernel(const float2* __restrict__ spec, float* __restrict__ x) {
    const int r = blockIdx.x * 256 + (threadIdx.x >> 2);
    const admm::quad::Lane L = admm::quad::lane_of(threadIdx.x);
    const float2* in = spec + (size_t)r * 128 + 32 * L.p;
    float2 S[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) S[k] = in[k];
    admm::quad::line_inverse(S, L);
    float2* row = reinterpret_cast<float2*>(x + (size_t)r * 256) + L.q;
#pragma unroll
    for (int m = 0; m < 32; ++m) row[4 * m] = S[m];
}

// timing: `reps` inverse + forward round trips of every line in registers (scaled by 1/256 each time)
__global__ __launch_bounds__(1024) void quad_bench_kernel(const float* __restrict__ x, float* __restrict__ y, int reps) {
    const int r = blockIdx.x * 256 + (threadIdx.x >> 2);
    const admm::quad::Lane L = admm::quad::lane_of(threadIdx.x);
    const float2* row = reinterpret_cast<const float2*>(x + (size_t)r * 256) + L.q;
    float2 S[32];
#pragma unroll
    for (int m = 0; m < 32; ++m) S[m] = row[4 * m];
    for (int i = 0; i < reps; ++i) {
        admm::quad::line_forward(S, L);
        admm::quad::line_inverse(S, L);
#pragma unroll
        for (int m = 0; m < 32; ++m) S[m] = admm::cscale(S[m], 1.0f / 256.0f);
    }
    float2* o = reinterpret_cast<float2*>(y + (size_t)r * 256) + L.q;
#pragma unroll
    for (int m = 0; m < 32; ++m) o[4 * m] = S[m];
}
__global__ __launch_bounds__(512) void pair_bench_kernel(const float* __restrict__ x, float* __restrict__ y, int reps) {
    const int r = blockIdx.x * 256 + (threadIdx.x >> 1);
    const bool hb = threadIdx.x & 1;
    const float2* row = reinterpret_cast<const float2*>(x + (size_t)r * 256) + (hb ? 1 : 0);
    float2 S[64];
#pragma unroll
    for (int n = 0; n < 64; ++n) S[n] = row[2 * n];
    for (int i = 0; i < reps; ++i) {
        admm::line_forward_pair(S, hb);
        admm::line_inverse_pair(S, hb);
#pragma unroll
        for (int n = 0; n < 64; ++n) S[n] = admm::cscale(S[n], 1.0f / 256.0f);
    }
    float2* o = reinterpret_cast<float2*>(y + (size_t)r * 256) + (hb ? 1 : 0);
#pragma unroll
    for (int n = 0; n < 64; ++n) o[2 * n] = S[n];
}

}  // namespace

template <int MODE, bool PSF = false>
int plane_debug(const float* y, float* x, const float* Cf, const float* C0b, float* hln, float* sln, float tau,
                       float rho, int K, int planes, float* dbg, const float* Gf = nullptr, const float* G0b = nullptr) {
    namespace pk = admm::plane;
    static float* prm = nullptr;   // the kernel reads {tau, rho} from device memory (setup_kernel's block)
    if (!prm && hipMalloc(&prm, 16) != hipSuccess) return -4;
    const float hp[4] = {tau, rho, 0.f, 0.f};
    if (hipMemcpy(prm, hp, sizeof(hp), hipMemcpyHostToDevice) != hipSuccess) return -4;
    (void)hipFuncSetAttribute((const void*)pk::plane256_kernel<PSF, MODE>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)pk::kLdsBytes);
    hipLaunchKernelGGL((pk::plane256_kernel<PSF, MODE>), dim3(planes), dim3(pk::kPT), pk::kLdsBytes, 0, y, x, Cf, C0b,
                       reinterpret_cast<const float2*>(Gf), reinterpret_cast<const float2*>(G0b),
                       reinterpret_cast<float2*>(hln), reinterpret_cast<float4*>(sln), prm, K,
                       reinterpret_cast<float2*>(dbg), 0);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -4;
}

extern "C" {
// Where a recording keeps its trajectory (tests read the GPU forward's own s_k / |s_k| back, to hold the
// gradient oracle's prox masks at the GPU's, tests/test_gpu_adjoint_masked.py): byte offsets from the
// 256-B aligned workspace base of s_1..s_{K-1} and (isotropic) of the batch norms |s_k|.
int devtest_recording_offsets(int M, int N, int P, int B, int kh, int maxit, int want_h, int iso, size_t* traj_s,
                              size_t* traj_n) {
    const admm::layout::BwdHead b =
        admm::layout::bwd_head(M, N, (size_t)P * B, kh, maxit, want_h != 0, iso != 0);
    *traj_s = b.traj_s;
    *traj_n = b.traj_n;
    return 0;
}
// The reverse sweep's h_bar intermediates (tools/hbar_paths.py: which of h_bar's two cancelling paths carries
// the error): byte offsets of Vsum (planes x M x N fp32), Q (fp64 (M/2+1) x N, after the plane sum), the path
// through H^T y and the path through C (kh x kw fp64 each), from the library's own backward layout.
int devtest_hbar_offsets(int M, int N, int P, int B, int kh, int kw, int maxit, size_t* out4) {
    const admm_capi::BwdLayout b = admm_capi::make_bwd_layout(M, N, (size_t)P * B, kh, kw, maxit, true, false, false);
    out4[0] = b.vsum;
    out4[1] = b.Q;
    out4[2] = b.hcorr;
    out4[3] = b.hA;
    return 0;
}
// fused plane kernel (no PSF) with per-phase dumps of plane 0: dbg holds (4K) x 64 x 512 float2.
// Cf/C0b must be the lane-native tables; hln/sln workspaces as in admm_capi.hip.
int devtest_plane_debug(const float* y, float* x, const float* Cf, const float* C0b, float* hln, float* sln, float tau,
                        float rho, int K, int planes, float* dbg) {
    return plane_debug<1>(y, x, Cf, C0b, hln, sln, tau, rho, K, planes, dbg);
}
// timing: dbg = planes x 8 waves x 512 u64 clock stamps (slot 4k-3.. as above, 256+k after column half 0)
int devtest_plane_timing(const float* y, float* x, const float* Cf, const float* C0b, float* hln, float* sln,
                         float tau, float rho, int K, int planes, float* dbg) {
    return plane_debug<2>(y, x, Cf, C0b, hln, sln, tau, rho, K, planes, dbg);
}
// workgroup start / end only (slots 508 / 509 of wave 0, s_memrealtime), the product kernel otherwise
int devtest_plane_wg_times(const float* y, float* x, const float* Cf, const float* C0b, float* hln, float* sln,
                           float tau, float rho, int K, int planes, float* dbg) {
    return plane_debug<3>(y, x, Cf, C0b, hln, sln, tau, rho, K, planes, dbg);
}
#ifdef PLANE_TS
int devtest_plane_ts_set(unsigned long long* buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(admm::plane::g_plane_ts), &buf, sizeof(buf)) == hipSuccess ? 0 : -4;
}
#endif
int devtest_plane_tables(const float* Ct, float* Cf, float* C0b) {
    namespace pk = admm::plane;
    hipLaunchKernelGGL(pk::tables_kernel, dim3(pk::kTab / 256), dim3(256), 0, 0, Ct, nullptr, Cf, C0b, nullptr, nullptr);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -4;
}
// PSF variant: Gt = conj(Sigma_c)/(MN) as float2[256][129]; Gf = kTab float2, G0b = 256 float2
int devtest_plane_tables_psf(const float* Ct, const float* Gt, float* Cf, float* C0b, float* Gf, float* G0b) {
    namespace pk = admm::plane;
    hipLaunchKernelGGL(pk::tables_kernel, dim3(pk::kTab / 256), dim3(256), 0, 0, Ct, reinterpret_cast<const float2*>(Gt),
                       Cf, C0b, reinterpret_cast<float2*>(Gf), reinterpret_cast<float2*>(G0b));
    return hipDeviceSynchronize() == hipSuccess ? 0 : -4;
}
int devtest_plane_debug_psf(const float* y, float* x, const float* Cf, const float* C0b, const float* Gf,
                            const float* G0b, float* hln, float* sln, float tau, float rho, int K, int planes,
                            float* dbg) {
    return plane_debug<1, true>(y, x, Cf, C0b, hln, sln, tau, rho, K, planes, dbg, Gf, G0b);
}
// rows must be a multiple of 256; device pointers; synchronous
int devtest_pair_forward(const float* x, float* spec, int rows) {
    pair_fwd_kernel<<<rows / 256, 512>>>(x, reinterpret_cast<float2*>(spec));
    return hipDeviceSynchronize() == hipSuccess ? 0 : -4;
}
int devtest_quad_forward(const float* x, float* spec, int rows) {
    quad_fwd_kernel<<<rows / 256, 1024>>>(x, reinterpret_cast<float2*>(spec));
    return hipDeviceSynchronize() == hipSuccess ? 0 : -4;
}
int devtest_quad_inverse(const float* spec, float* x, int rows) {
    quad_inv_kernel<<<rows / 256, 1024>>>(reinterpret_cast<const float2*>(spec), x);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -4;
}
// line-transform round trips, lane-quad (quad = 1) or lane-pair layout; returns kernel ms through *ms
int devtest_line_bench(const float* x, float* y, int rows, int reps, int quad, float* ms) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    if (quad) quad_bench_kernel<<<rows / 256, 1024>>>(x, y, reps);
    else pair_bench_kernel<<<rows / 256, 512>>>(x, y, reps);
    hipEventRecord(b);
    const bool ok = hipEventSynchronize(b) == hipSuccess;
    hipEventElapsedTime(ms, a, b);
    hipEventDestroy(a);
    hipEventDestroy(b);
    return ok ? 0 : -4;
}
int devtest_pair_inverse(const float* spec, float* x, int rows) {
    pair_inv_kernel<<<rows / 256, 512>>>(reinterpret_cast<const float2*>(spec), x);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -4;
}
}
