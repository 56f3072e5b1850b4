// admm_kernels.hip -- MI355X (gfx950) kernels for the ADMM TV-deconvolution solve.
//
// Replaces the per-iteration CUFFT / cuDNN / broadcast chain of tvd_fft_gpu
// (/root/reference/src/ops/ops.jl:99-178) with two fused passes per iteration:
//
//   COLUMN pass  (ops.jl:168: the dim2 half of rfft/irfft and the C .* scale)
//       spec[plane][j][k]  --FFT_j--> x C[k][kj] --IFFT_j-->  spec1[plane][j][k]      (in place OK)
//   LINE pass    (ops.jl:168-173 + the dim1 half of the transforms)
//       spec1 --irFFT_i--> x --D--> s = Dx + u --prox--> w = z-u --D^T--> v = H^T y + rho D^T w
//       --rFFT_i--> spec0, and s written back (ping-pong) as the only per-pixel ADMM state.
//
// State compression: with s_k = Dx_k + u_{k-1}, the reference's z_k = ST(s_k) and
// u_k = s_k - z_k = clip(s_k, -tau, tau) are functions of s_k alone, so one 2-channel fp32 tensor
// replaces the reference's Dx, z and u (ops.jl:128-131).
//
// Half-spectrum packing: a line of M reals has M/2+1 bins; bins 0 and M/2 are real and share slot 0
// as (X[0], X[M/2]), so a line's spectrum is exactly M/2 complex (1 KiB at M = 256).  Rows k = 0 and
// k = M/2 of any multiplier used here are Hermitian in kj, so the column pass applies slot 0 as
//   R[kj] = (m0+mL)/2 Z[kj] + (m0-mL)/2 conj(Z[-kj]).
//
// Real <-> half-length complex: z[n] = x[2n] + i x[2n+1]; Z = FFT_{M/2}(z);
//   X[k] = E[k] + W_M^k O[k], E = (Z[k] + conj Z[L-k])/2, O = (Z[k] - conj Z[L-k])/(2i).
// All transforms are unnormalised; 1/(M N) is folded into the multiplier tables.
//
// H^T y (ops.jl:71-81) is evaluated ONCE (the reference re-evaluates it every iteration and gets the
// same array) and spectrally: H^T y = F^-1[ conj(Sigma_c) F y ] with Sigma_c the spectrum of the
// centred PSF -- the same line/column kernels with a complex multiplier.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fft_reg.hpp"
#include "plane_api.hpp"
#include "scalar_src.hpp"

namespace admm {

constexpr int kThreads = 256;
// Several branches in one grid (admm_launch.hip launch_forward_multi below the plane-count rule): grid plane
// q = i ppb + loc is branch i's solve of input plane loc; its output plane is the chcat position
// (plane::branch_of).  The 2-pass kernels take per-branch C tables tab_f floats apart, {tau, rho, lambda}
// blocks prm_f floats apart and per-branch M x N maps (f, |s|, R) M N floats apart.  nbr = 1: one solve.
using plane::Branches;
using plane::BranchOf;
using plane::branch_of;
constexpr Branches kOneSolve{1, 1, 1, 0u, 0u};
// source / destination plane of a line transform: the grid plane, the shared input plane, or the chcat plane
enum PlaneMap { kMapGrid = 0, kMapIn = 1, kMapOut = 2 };
__device__ __forceinline__ size_t map_plane(const Branches& br, int map, size_t plane) {
    if (map == kMapGrid || br.nbr == 1) return plane;
    const BranchOf bo = branch_of(br, plane);
    return map == kMapIn ? bo.in_plane : bo.out_plane;
}
constexpr int kSetupPsfLds = 4096;   // PSF taps the setup kernel stages in LDS (larger PSFs are read from global)
constexpr int kSetupSplit = 4;       // setup_kernel lanes per spectral bin

// XCD-aware block order (2-D grid (x, y) -> logical (x, y)).  Workgroups are dealt round-robin over
// the 8 XCDs, each with its own L2 (MI355X_MICROARCH.md, workgroup dispatch): the bijective remap
// gives each XCD a contiguous run of logical blocks, so neighbours that share cache lines (column
// slots 32 B apart at N = 512, the halo lines of line tiles) hit the same L2.  Speed only.
struct XBlk {
    int x, y;
};
__device__ __forceinline__ XBlk xcd_block() {
#ifdef ADMM_NO_XCD_SWIZZLE
    return {(int)blockIdx.x, (int)blockIdx.y};
#else
    const unsigned nx = gridDim.x, n = nx * gridDim.y;
    const unsigned orig = blockIdx.x + nx * blockIdx.y;
    const unsigned q = n / 8, r = n % 8, g = orig % 8;
    const unsigned id = (g < r ? g * (q + 1) : r * (q + 1) + (g - r) * q) + orig / 8;
    return {(int)(id % nx), (int)(id / nx)};
#endif
}

// ----------------------------------------------------------------------------------------------
// setup: twiddle tables and multiplier tables, built in fp64 (ops.jl:22-37)
//   Ct[kj][k] = 1/(MN) / (|Sigma|^2 + rho(|Lx|^2 + |Ly|^2))     k = 0..M/2  (transposed: k fastest)
//   Gt[kj][k] = 1/(MN) * conj(Sigma_centred)                      (only with a PSF)
// ----------------------------------------------------------------------------------------------
// Where the solve's lambda and rho come from: device pointers (the reference's 1-element CuArrays,
// `tvd_fft(y, λ::CGPUArray, ρ::CGPUArray, ...)`, ops.jl:99,181 -- read on the device, no host sync)
// or, when a pointer is NULL, the host value.  setup_kernel resolves them once into the
// workspace's scalar block prm = {tau = lambda / rho (fp32, ops.jl:20), rho, lambda}; every later
// kernel of the solve reads prm, and a recording's replay reuses the block the recording resolved.
__device__ __forceinline__ float src_lam(const ScalarSrc& sc) { return sc.lam ? *sc.lam : sc.lam_v; }
__device__ __forceinline__ float src_rho(const ScalarSrc& sc) { return sc.rho ? *sc.rho : sc.rho_v; }
__device__ __forceinline__ void write_prm(const ScalarSrc& sc, float* prm) {
    const float lam = src_lam(sc), rho = src_rho(sc);
    prm[0] = lam / rho;
    prm[1] = rho;
    prm[2] = lam;
}
__global__ __launch_bounds__(kThreads) void setup_kernel(float2* __restrict__ twM, float2* __restrict__ twN,
                                                         float* __restrict__ Ct, float2* __restrict__ Gt,
                                                         const float* __restrict__ h, int kh, int kw, int M,
                                                         int N, ScalarSrc sc, float* __restrict__ prm,
                                                         double2* __restrict__ SigT) {
    const float rho = src_rho(sc);
    if (blockIdx.x == 0 && threadIdx.x == 0) write_prm(sc, prm);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    double2* tM = reinterpret_cast<double2*>(smem_raw);  // exp(-2 pi i t / M)
    double2* tN = tM + M;                                // exp(-2 pi i t / N)
    for (int t = threadIdx.x; t < M; t += blockDim.x) {
        double s, c;
        sincospi(-2.0 * (double)t / (double)M, &s, &c);
        tM[t] = make_double2(c, s);
    }
    for (int t = threadIdx.x; t < N; t += blockDim.x) {
        double s, c;
        sincospi(-2.0 * (double)t / (double)N, &s, &c);
        tN[t] = make_double2(c, s);
    }
    // the PSF in LDS when it has at most kSetupPsfLds taps (the launch sizes the LDS for it): each bin reads every
    // tap, and a global load per tap waited on inside the runtime-length loop cost an L2 latency per term
    const bool psf_lds = kh * kw <= kSetupPsfLds;
    float* hl = reinterpret_cast<float*>(tN + N);
    if (psf_lds)
        for (int t = threadIdx.x; t < kh * kw; t += blockDim.x) hl[t] = h[t];
    const float* hs = psf_lds ? hl : h;
    __syncthreads();
    if (blockIdx.x == 0) {
        for (int t = threadIdx.x; t < M; t += blockDim.x) twM[t] = make_float2((float)tM[t].x, (float)tM[t].y);
        for (int t = threadIdx.x; t < N; t += blockDim.x) twN[t] = make_float2((float)tN[t].x, (float)tN[t].y);
    }
    const int L = M / 2;
    const int H = L + 1;
    const int nbins = H * N;
    const double inv_mn = 1.0 / ((double)M * (double)N);
    const int padd = (kh - 1) / 2, padr = (kw - 1) / 2;
    // kSetupSplit lanes per bin, each summing the PSF columns b = sub, sub + kSetupSplit, ...; the partial sums meet
    // in a fixed xor-shuffle order.  (One lane per bin left 129 blocks at 256^2, each thread a 225-term dependent
    // fp64 chain: 17.7 us of every c2 call.)
    const int split = kh > 0 ? kSetupSplit : 1;
    const int sub = threadIdx.x & (split - 1);
    for (int qq = blockIdx.x * blockDim.x + threadIdx.x; qq < nbins * split; qq += gridDim.x * blockDim.x) {
        const int q = qq / split;   // the split lanes of a bin are neighbours in one iteration
        const int kj = q / H;   // dim2 frequency
        const int k = q - kj * H;  // dim1 frequency 0..L
        double s2 = 1.0;
        if (kh > 0) {
            double re = 0.0, im = 0.0;
            // table indices (b kj) mod N and (a k) mod M advanced by one addition and one conditional
            // subtraction (kj < N, k < M) instead of an integer division per term: the same entries
            const int bstep = (int)(((long long)split * kj) % N);
            int ib = (int)(((long long)sub * kj) % N);
            for (int b = sub; b < kw; b += split) {
                const double2 eb = tN[ib];
                double gr = 0.0, gi = 0.0;
                int ia = 0;
                for (int a = 0; a < kh; ++a) {
                    const double w = (double)hs[b * kh + a];
                    const double2 ea = tM[ia];
                    gr += w * ea.x;
                    gi += w * ea.y;
                    ia += k;
                    if (ia >= M) ia -= M;
                }
                re += gr * eb.x - gi * eb.y;
                im += gr * eb.y + gi * eb.x;
                ib += bstep;
                if (ib >= N) ib -= N;
            }
#pragma unroll
            for (int o = 1; o < kSetupSplit; o <<= 1) {
                re += __shfl_xor(re, o);
                im += __shfl_xor(im, o);
            }
            s2 = re * re + im * im;
            if (sub != 0) continue;
            if (SigT) SigT[q] = make_double2(re, im);   // top-left PSF spectrum (backward h_bar)
            // centred spectrum: Sigma_c = Sigma * exp(+2 pi i (padd k/M + padr kj/N)); store conj / (MN)
            const double2 pa = tM[(padd * k) % M];
            const double2 pb = tN[(padr * kj) % N];
            const double pr = pa.x * pb.x - pa.y * pb.y, pi = pa.x * pb.y + pa.y * pb.x;  // exp(-i phi)
            // Sigma_c = Sigma * conj(p);  conj(Sigma_c) = conj(Sigma) * p
            const double cr = re * pr + im * pi;
            const double ci = re * pi - im * pr;
            Gt[q] = make_float2((float)(cr * inv_mn), (float)(ci * inv_mn));
        }
        if (sub != 0) continue;
        const double sx = sinpi((double)kj / (double)N), sy = sinpi((double)k / (double)M);
        const double lap = 4.0 * sx * sx + 4.0 * sy * sy;   // |Lx|^2 + |Ly|^2 (ops.jl:35-36)
        Ct[q] = (float)(inv_mn / (s2 + (double)rho * lap));
    }
}

// ----------------------------------------------------------------------------------------------
// line helpers
// ----------------------------------------------------------------------------------------------
// Z[n] of the inverse half-length transform, from the packed half spectrum X of one line (LDS)
template <int L>
__device__ __forceinline__ float2 unpack_z(const float2* __restrict__ Xl, int n, const float2* __restrict__ tw) {
    if (n == 0) {
        const float2 p = Xl[0];  // (X[0], X[M/2]), both real
        return make_float2(p.x + p.y, p.x - p.y);
    }
    const float2 xk = Xl[n];
    const float2 xm = cconj(Xl[L - n]);
    const float2 e = cadd(xk, xm);
    const float2 o = cmul(csub(xk, xm), cconj(tw[n]));  // * W_M^{-n}
    return make_float2(e.x - o.y, e.y + o.x);            // E + i O
}

// packed half-spectrum bin k of a real line from its half-length transform Z (LDS)
template <int L>
__device__ __forceinline__ float2 pack_x(const float2* __restrict__ Zl, int k, const float2* __restrict__ tw) {
    if (k == 0) {
        const float2 z0 = Zl[0];
        return make_float2(z0.x + z0.y, z0.x - z0.y);
    }
    const float2 zk = Zl[k];
    const float2 zm = cconj(Zl[L - k]);
    const float2 e = cscale(cadd(zk, zm), 0.5f);
    const float2 d = csub(zk, zm);
    const float2 o = make_float2(0.5f * d.y, -0.5f * d.x);  // d / (2i)
    return cadd(e, cmul(tw[k], o));
}

template <int L>
__device__ __forceinline__ void pack_store(const float2* __restrict__ Z, float2* __restrict__ out_plane, int j0,
                                           int nlines, int N, const float2* __restrict__ tw) {
    for (int idx = threadIdx.x; idx < nlines * L; idx += blockDim.x) {
        const int t = idx / L;
        const int k = idx - t * L;
        out_plane[(size_t)((j0 + t) & (N - 1)) * L + k] = pack_x<L>(Z + t * L, k, tw);
    }
}

template <int L>
__device__ __forceinline__ void load_lines(const float2* __restrict__ plane, float2* __restrict__ dst, int j0,
                                           int nlines, int N) {
    const float4* src4 = reinterpret_cast<const float4*>(plane);
    float4* d4 = reinterpret_cast<float4*>(dst);
    constexpr int L2 = L / 2;  // float4 per line
    for (int idx = threadIdx.x; idx < nlines * L2; idx += blockDim.x) {
        const int t = idx / L2;
        const int q = idx - t * L2;
        d4[idx] = src4[(size_t)((j0 + t) & (N - 1)) * L2 + q];
    }
}

__device__ __forceinline__ float clipf(float s, float tau) { return fminf(fmaxf(s, -tau), tau); }
// w = z - u for z = ST(s, tau), u = s - z  (ops.jl:9, :171-173)
__device__ __forceinline__ float prox_w(float s, float tau) {
    return fabsf(s) > tau ? s - copysignf(2.0f * tau, s) : -s;
}

// ----------------------------------------------------------------------------------------------
// LINE_FWD: rFFT along dim1 of T real lines of a plane (y or any real field) -> packed spectrum
// ----------------------------------------------------------------------------------------------
template <int L, int T>
__global__ __launch_bounds__(kThreads) void line_fwd_kernel(const float* __restrict__ src, float2* __restrict__ spec,
                                                            const float2* __restrict__ twM, int N,
                                                            Branches br = kOneSolve, int map = kMapGrid) {
    constexpr int M = 2 * L;
    constexpr int P = Plan<L>::P;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float2* tw = reinterpret_cast<float2*>(smem_raw);
    float2* X = tw + M;
    float2* Bf = X + T * L;
    const XBlk xb = xcd_block();
    const int plane = xb.y;
    const int j0 = xb.x * T;
    for (int t = threadIdx.x; t < M; t += blockDim.x) tw[t] = twM[t];
    __syncthreads();
    const float2* sp = reinterpret_cast<const float2*>(src + map_plane(br, map, plane) * N * M);
    auto gload = [&](int f, int n) { return sp[(size_t)(j0 + f) * L + n]; };
    float2* Z = (P == 2) ? Bf : X;
    fft_plan<L, true, false, 2>(T, tw, X, Bf, L, gload, LdsIO{Z, L});
    __syncthreads();
    pack_store<L>(Z, spec + (size_t)plane * N * L, j0, T, N, tw);
}

// ----------------------------------------------------------------------------------------------
// LINE_INV: irFFT along dim1 of T lines -> real lines (final x, or H^T y during setup)
// ----------------------------------------------------------------------------------------------
template <int L, int T>
__global__ __launch_bounds__(kThreads) void line_inv_kernel(const float2* __restrict__ spec, float* __restrict__ dst,
                                                            const float2* __restrict__ twM, int N,
                                                            Branches br = kOneSolve, int map = kMapGrid) {
    constexpr int M = 2 * L;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float2* tw = reinterpret_cast<float2*>(smem_raw);
    float2* X = tw + M;
    float2* Bf = X + T * L;
    const XBlk xb = xcd_block();
    const int plane = xb.y;
    const int j0 = xb.x * T;
    for (int t = threadIdx.x; t < M; t += blockDim.x) tw[t] = twM[t];
    load_lines<L>(spec + (size_t)plane * N * L, X, j0, T, N);
    __syncthreads();
    float2* dp = reinterpret_cast<float2*>(dst + map_plane(br, map, plane) * N * M);
    auto uload = [&](int f, int n) { return unpack_z<L>(X + f * L, n, tw); };
    auto gstore = [&](int f, int n, float2 v) { dp[(size_t)(j0 + f) * L + n] = v; };
    fft_plan<L, false, true, 2>(T, tw, Bf, X, L, uload, gstore);
}

// ----------------------------------------------------------------------------------------------
// COLUMN pass: KB consecutive slots of one plane; FFT along dim2 (NN points), multiply, inverse.
// Forward plan, then the reversed plan for the inverse, so the forward's last pass and the inverse's
// first pass touch the same points in the same thread: they run back to back in registers with the
// multiply between (one LDS round trip saved).  One LDS buffer, in-place passes (read, barrier,
// write); requires KB * NN / R <= blockDim for every radix R of the plan (host guarantees).
//   MUL = 0: real multiplier Ct (the ADMM x-update / its adjoint A^-1), scaled by cs
//   MUL = 1: complex multiplier Gt = conj(Sigma_c)/(MN)   (H^T y setup)
//   MUL = 2: conj(Gt) = Sigma_c/(MN)                       (y_bar = H vbar_sum in the backward)
//   SAVE   : also store the forward dim-2 spectrum (before the multiply) to vsave (trajectory for h_bar)
//   ACCQ   : accumulate Q[kj][k] += Re(conj(G) V) against the saved forward spectrum (adjoint, h_bar), in fp64:
//            K terms per bin, later scaled by C^2 in hbarA_kernel
//   YH     : the spectrum of H^T y enters in the spectral domain (DESIGN.md s1 "H^T y in the spectrum"):
//            YH_STORE: forward transform, x Gt (conj(Sigma_c)/(MN); none when Gt is NULL), x cs, stored to yh as
//                      the plane's 2-D packed spectrum Y_h = F(H^T y) -- no inverse, dst untouched;
//            YH_ADD:   yh added to the forward spectrum (before the mirror staging, SAVE and the multiply), so the
//                      per-iteration transforms carry only rho D^T w and H^T y never passes an fp32 FFT again
// ----------------------------------------------------------------------------------------------
enum { YH_NONE = 0, YH_STORE = 1, YH_ADD = 2 };
// The body takes the block's (slot block, plane) explicitly (a persistent kernel can run it too: the round-5 team
// launch, tools/variants/team512.patch); column_kernel is the one-launch-per-pass form.
template <int NN, int MUL, bool SAVE, bool ACCQ, int NT = kThreads, int YH = YH_NONE>
__device__ __forceinline__ void column_body(XBlk xb, const float2* src, float2* dst, const float* __restrict__ Ct,
                                            const float2* __restrict__ Gt, const float2* __restrict__ twN, int L,
                                            int KB, float cs, float2* __restrict__ vsave, double* __restrict__ Qp,
                                            float2* __restrict__ yh = nullptr) {
    constexpr bool CPLX = MUL != 0;
    constexpr int FS = NN + 1;  // per-transform LDS stride (odd: conflict-free slot-major stores)
    constexpr int P = Plan<NN>::P;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float2* tw = reinterpret_cast<float2*>(smem_raw);
    float2* S0 = tw + NN;        // slot-0 spectrum for the mirror term
    float2* buf = S0 + NN;
    const int plane = xb.y;
    const int k0 = xb.x * KB;
    const int H = L + 1;
    const float2* gsrc = src + (size_t)plane * NN * L + k0;
    float2* gdst = dst + (size_t)plane * NN * L + k0;
    for (int t = threadIdx.x; t < NN; t += blockDim.x) tw[t] = twN[t];
    __syncthreads();
    const int tid = threadIdx.x;
    // ---- forward pass 0: global -> regs -> LDS   (thread = (j, f), slot f fastest) ----
    {
        constexpr int R = plan_radix<NN, 0, false>();
        constexpr int Q = NN / R;
        if (tid < KB * Q) {
            const int f = tid % KB, j = tid / KB;
            float2 v[R];
#pragma unroll
            for (int r = 0; r < R; ++r) v[r] = gsrc[(size_t)(j + r * Q) * L + f];
            if constexpr (P == 1) {
                // single-pass plan: handled below in the fused step (no LDS staging needed)
            }
            fly_core<NN, R, 0, false, 1>(v, j, tw);
            const int o = out_base<NN, R, 0>(j);
#pragma unroll
            for (int r = 0; r < R; ++r) buf[f * FS + o + r] = v[r];
        }
    }
    __syncthreads();
    if constexpr (P == 3) {   // forward middle pass, in place
        constexpr int R = plan_radix<NN, 1, false>();
        constexpr int LG = plan_lgns<NN, 1, false>();
        constexpr int Q = NN / R;
        float2 v[R];
        const int f = tid % KB, j = tid / KB;
        const bool act = tid < KB * Q;
        if (act) {
#pragma unroll
            for (int r = 0; r < R; ++r) v[r] = buf[f * FS + j + r * Q];
        }
        __syncthreads();
        if (act) {
            fly_core<NN, R, LG, false, 1>(v, j, tw);
            const int o = out_base<NN, R, LG>(j);
#pragma unroll
            for (int r = 0; r < R; ++r) buf[f * FS + o + r * (1 << LG)] = v[r];
        }
        __syncthreads();
    }
    // ---- fused: forward last pass -> multiply -> inverse first pass ----
    {
        constexpr int PL = P - 1;
        constexpr int R = plan_radix<NN, PL, false>();
        constexpr int LG = plan_lgns<NN, PL, false>();
        constexpr int Q = NN / R;   // == Ns of the last pass: outputs at j + r*Q
        float2 v[R];
        const int f = tid % KB, j = tid / KB;
        const bool act = tid < KB * Q;
        const bool mirror = (k0 == 0);  // block-uniform
        if (act) {
            if constexpr (P > 1) {
#pragma unroll
                for (int r = 0; r < R; ++r) v[r] = buf[f * FS + j + r * Q];
                fly_core<NN, R, LG, false, 1>(v, j, tw);
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) v[r] = buf[f * FS + j + r * Q];
            }
            if constexpr (YH == YH_ADD) {   // + F(H^T y): before the slot-0 staging, the mirror reads the sum
                const float2* yp = yh + (size_t)plane * NN * L + k0 + f;
#pragma unroll
                for (int r = 0; r < R; ++r) v[r] = cadd(v[r], yp[(size_t)(j + r * Q) * L]);
            }
            if (mirror && f == 0) {
#pragma unroll
                for (int r = 0; r < R; ++r) S0[j + r * Q] = v[r];
            }
        }
        __syncthreads();
        if (act) {
            const int s = k0 + f;
            if constexpr (SAVE) {
                float2* vs = vsave + (size_t)plane * NN * L + k0;
#pragma unroll
                for (int r = 0; r < R; ++r) vs[(size_t)(j + r * Q) * L + f] = cscale(v[r], cs);
            }
            if constexpr (ACCQ) {
                const float2* vs = vsave + (size_t)plane * NN * L;
                double* qp = Qp + (size_t)plane * NN * H;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int kj = j + r * Q;
                    const float2 gv = v[r];
                    const float2 vv = vs[(size_t)kj * L + s];
                    if (mirror && f == 0) {
                        // separate the packed pair: A = (Z + conj Z(-kj))/2, B = (Z - conj Z(-kj))/(2i)
                        const int km = (NN - kj) & (NN - 1);
                        const float2 gm = cconj(S0[km]);
                        const float2 vm = cconj(vs[(size_t)km * L]);
                        const float2 ga = cscale(cadd(gv, gm), 0.5f), va = cscale(cadd(vv, vm), 0.5f);
                        const float2 gd = csub(gv, gm), vd = csub(vv, vm);
                        const float2 gb = make_float2(0.5f * gd.y, -0.5f * gd.x);
                        const float2 vb = make_float2(0.5f * vd.y, -0.5f * vd.x);
                        qp[(size_t)kj * H] += (double)ga.x * va.x + (double)ga.y * va.y;
                        qp[(size_t)kj * H + L] += (double)gb.x * vb.x + (double)gb.y * vb.y;
                    } else {
                        qp[(size_t)kj * H + s] += (double)gv.x * vv.x + (double)gv.y * vv.y;
                    }
                }
            }
            // (YH_STORE without a PSF: Y_h = F y, no multiplier)
            if (YH != YH_STORE || Gt != nullptr)
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int kj = j + r * Q;
                if (mirror && f == 0) {
                    const float2 zm = cconj(S0[(NN - kj) & (NN - 1)]);
                    if constexpr (CPLX) {
                        float2 m0 = Gt[(size_t)kj * H], mL = Gt[(size_t)kj * H + L];
                        if constexpr (MUL == 2) { m0 = cconj(m0); mL = cconj(mL); }
                        const float2 a = cscale(cadd(m0, mL), 0.5f), b = cscale(csub(m0, mL), 0.5f);
                        v[r] = cadd(cmul(a, v[r]), cmul(b, zm));
                    } else {
                        const float c0 = Ct[(size_t)kj * H], cL = Ct[(size_t)kj * H + L];
                        v[r] = cadd(cscale(v[r], 0.5f * cs * (c0 + cL)), cscale(zm, 0.5f * cs * (c0 - cL)));
                    }
                } else {
                    if constexpr (MUL == 2) {
                        v[r] = cmul(v[r], cconj(Gt[(size_t)kj * H + s]));
                    } else if constexpr (CPLX) {
                        v[r] = cmul(v[r], Gt[(size_t)kj * H + s]);
                    } else {
                        v[r] = cscale(v[r], cs * Ct[(size_t)kj * H + s]);
                    }
                }
            }
            if constexpr (YH == YH_STORE) {   // Y_h = cs Gt F y: stored, no inverse
                float2* yp = yh + (size_t)plane * NN * L + k0 + f;
#pragma unroll
                for (int r = 0; r < R; ++r) yp[(size_t)(j + r * Q) * L] = cscale(v[r], cs);
            } else {
            // inverse first pass (reversed plan: radix R, Ns = 1) reads exactly j + r*Q
            dft<R, true>(v);
            if constexpr (P == 1) {
#pragma unroll
                for (int r = 0; r < R; ++r) gdst[(size_t)(j * R + r) * L + f] = v[r];
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) buf[f * FS + j * R + r] = v[r];
            }
            }
        }
        if constexpr (YH == YH_STORE) return;   // block-uniform
        __syncthreads();
    }
    if constexpr (P == 3) {   // inverse middle pass (reversed plan pass 1), in place
        constexpr int R = plan_radix<NN, 1, true>();
        constexpr int LG = plan_lgns<NN, 1, true>();
        constexpr int Q = NN / R;
        float2 v[R];
        const int f = tid % KB, j = tid / KB;
        const bool act = tid < KB * Q;
        if (act) {
#pragma unroll
            for (int r = 0; r < R; ++r) v[r] = buf[f * FS + j + r * Q];
        }
        __syncthreads();
        if (act) {
            fly_core<NN, R, LG, true, 1>(v, j, tw);
            const int o = out_base<NN, R, LG>(j);
#pragma unroll
            for (int r = 0; r < R; ++r) buf[f * FS + o + r * (1 << LG)] = v[r];
        }
        __syncthreads();
    }
    if constexpr (P > 1) {    // inverse last pass: LDS -> regs -> global
        constexpr int PL = P - 1;
        constexpr int R = plan_radix<NN, PL, true>();
        constexpr int LG = plan_lgns<NN, PL, true>();
        constexpr int Q = NN / R;
        if (tid < KB * Q) {
            const int f = tid % KB, j = tid / KB;
            float2 v[R];
#pragma unroll
            for (int r = 0; r < R; ++r) v[r] = buf[f * FS + j + r * Q];
            fly_core<NN, R, LG, true, 1>(v, j, tw);
            const int o = out_base<NN, R, LG>(j);
#pragma unroll
            for (int r = 0; r < R; ++r) gdst[(size_t)(o + r * (1 << LG)) * L + f] = v[r];
        }
    }
}

template <int NN, int MUL, bool SAVE, bool ACCQ, int NT = kThreads, int YH = YH_NONE>
__global__ __launch_bounds__(NT) void column_kernel(const float2* src, float2* dst, const float* __restrict__ Ct,
                                                    const float2* __restrict__ Gt, const float2* __restrict__ twN, int L,
                                                    int KB, float cs, float2* __restrict__ vsave,
                                                    double* __restrict__ Qp, Branches br = kOneSolve,
                                                    float2* __restrict__ yh = nullptr) {
    const XBlk xb = xcd_block();
    column_body<NN, MUL, SAVE, ACCQ, NT, YH>(xb, src, dst, Ct + (size_t)branch_of(br, xb.y).i * br.tab_f, Gt, twN, L,
                                             KB, cs, vsave, Qp, yh);
}

// ----------------------------------------------------------------------------------------------
// LINE pass (iterations 1..K-1): T output lines + 1 halo line on each side.
// ----------------------------------------------------------------------------------------------
template <int L, int T, int NT = kThreads>
__device__ __forceinline__ void line_body(XBlk xb, const float2* __restrict__ spec1, float2* __restrict__ spec0,
                                          const float* __restrict__ s_old, float* __restrict__ s_new,
                                          const float* __restrict__ hty, const float2* __restrict__ twM, int N,
                                          const float* __restrict__ prm, int s_zero, Branches br = kOneSolve) {
    constexpr int M = 2 * L;
    constexpr int M4 = M / 4;
    constexpr int TH = T + 2;
    constexpr int P = Plan<L>::P;
    constexpr int NE = (T + 1) * M4;                       // float4 items of the elementwise step
    constexpr int NIT = (NE + NT - 1) / NT;
    constexpr int RF = plan_radix<L, 0, true>();           // forward (reversed plan) first radix
    constexpr int QF = L / RF;
    constexpr int NITF = (T * QF + NT - 1) / NT;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float2* tw = reinterpret_cast<float2*>(smem_raw);
    float2* X = tw + M;           // TH lines
    float2* Bf = X + TH * L;      // TH lines
    float2* Cf = Bf + TH * L;     // TH lines (w1; 3rd ping-pong buffer for 3-pass plans)
    const int plane = xb.y;
    const int j0 = xb.x * T;
    const size_t MN = (size_t)M * N;
    const int tid = threadIdx.x;
    const float* so = s_old + (size_t)plane * 2 * MN;
    float* sn = s_new + (size_t)plane * 2 * MN;
    const BranchOf bo = branch_of(br, plane);   // several branches: H^T y = the shared input plane, own scalars
    // hty NULL: H^T y is added in the spectral domain by the column pass (YH_ADD); v = rho D^T w here
    const float* hp = hty ? hty + bo.in_plane * MN : nullptr;
    const float tau = prm[(size_t)bo.i * br.prm_f], rho = prm[(size_t)bo.i * br.prm_f + 1];   // (setup_kernel)

    // ---- issue every global load of the block up front -- except at 512-point lines (kJit): there the
    // s / H^T y loads go just before their use, which cuts the registers held across the irFFT (156 -> 88
    // VGPRs) so that 4-line blocks run 4 per CU (c4 line pass 1.173 -> 1.140 ms); at 256
    // points the early loads win (0.192 vs 0.201 ms) ----
    constexpr bool kJit = L == 256;
    for (int t = tid; t < M; t += NT) tw[t] = twM[t];
    load_lines<L>(spec1 + (size_t)plane * N * L, X, j0 - 1, TH, N);
    float4 pre0[NIT], pre1[NIT];
    auto load_s = [&] {
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int idx = tid + it * NT;
            const int t = idx / M4;
            const int i = (idx - t * M4) * 4;
            const size_t off = (size_t)((j0 + t) & (N - 1)) * M + i;
            pre0[it] = make_float4(0.f, 0.f, 0.f, 0.f);
            pre1[it] = pre0[it];
            if (!s_zero && idx < NE) {
                pre0[it] = *reinterpret_cast<const float4*>(so + off);
                if (t < T) pre1[it] = *reinterpret_cast<const float4*>(so + MN + off);
            }
        }
    };
    float2 preh[NITF][RF];
    auto load_h = [&] {
#pragma unroll
        for (int it = 0; it < NITF; ++it) {
            const int idx = tid + it * NT;
            const int f = idx / QF, j = idx - f * QF;
            if (hp && idx < T * QF) {
                const float2* hl = reinterpret_cast<const float2*>(hp + (size_t)(j0 + f) * M);
#pragma unroll
                for (int r = 0; r < RF; ++r) preh[it][r] = hl[j + r * QF];
            } else {
#pragma unroll
                for (int r = 0; r < RF; ++r) preh[it][r] = make_float2(0.f, 0.f);
            }
        }
    };
    if constexpr (!kJit) {
        load_s();
        load_h();
    }
    __syncthreads();

    // ---- irFFT along dim1 of TH lines: x (float view of the result buffer) ----
    auto uload = [&](int f, int n) { return unpack_z<L>(X + f * L, n, tw); };
    float2* Xr;
    if constexpr (P == 1) {
        Xr = Bf;
        fpass<L, L, 0, true, 2>(TH, tw, uload, LdsIO{Bf, L});
    } else if constexpr (P == 2) {
        Xr = X;  // pass 0: X -> Bf ; pass 1: Bf -> X
        fft_plan<L, false, true, 2>(TH, tw, Bf, Cf, L, uload, LdsIO{X, L});
    } else {
        Xr = Bf;  // X -> Bf -> Cf -> Bf
        plan_pass<L, 0, false, true, 2>(TH, tw, uload, LdsIO{Bf, L});
        __syncthreads();
        plan_pass<L, 1, false, true, 2>(TH, tw, LdsIO{Bf, L}, LdsIO{Cf, L});
        __syncthreads();
        plan_pass<L, 2, false, true, 2>(TH, tw, LdsIO{Cf, L}, LdsIO{Bf, L});
    }
    __syncthreads();
    const float* x = reinterpret_cast<const float*>(Xr);
    float* W0 = reinterpret_cast<float*>(Xr == X ? Bf : X);   // T+1 lines
    float* W1 = reinterpret_cast<float*>(Cf);                 // T lines
    if constexpr (kJit) {
        load_s();
        load_h();
    }

    // ---- s = Dx + u_old ; w = z - u   (ops.jl:169-173) ----
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
        const int idx = tid + it * NT;
        if (idx < NE) {
            const int t = idx / M4;
            const int i = (idx - t * M4) * 4;
            const size_t off = (size_t)((j0 + t) & (N - 1)) * M + i;
            const float4 xc = *reinterpret_cast<const float4*>(x + (t + 1) * M + i);
            const float4 xp = *reinterpret_cast<const float4*>(x + t * M + i);
            const float4 u0 = pre0[it];
            float4 s0;
            s0.x = (xc.x - xp.x) + clipf(u0.x, tau);
            s0.y = (xc.y - xp.y) + clipf(u0.y, tau);
            s0.z = (xc.z - xp.z) + clipf(u0.z, tau);
            s0.w = (xc.w - xp.w) + clipf(u0.w, tau);
            *reinterpret_cast<float4*>(W0 + t * M + i) =
                make_float4(prox_w(s0.x, tau), prox_w(s0.y, tau), prox_w(s0.z, tau), prox_w(s0.w, tau));
            if (t < T) {
                const float xl = x[(t + 1) * M + ((i - 1) & (M - 1))];
                const float4 u1 = pre1[it];
                float4 s1;
                s1.x = (xc.x - xl) + clipf(u1.x, tau);
                s1.y = (xc.y - xc.x) + clipf(u1.y, tau);
                s1.z = (xc.z - xc.y) + clipf(u1.z, tau);
                s1.w = (xc.w - xc.z) + clipf(u1.w, tau);
                *reinterpret_cast<float4*>(W1 + t * M + i) =
                    make_float4(prox_w(s1.x, tau), prox_w(s1.y, tau), prox_w(s1.z, tau), prox_w(s1.w, tau));
                *reinterpret_cast<float4*>(sn + off) = s0;
                *reinterpret_cast<float4*>(sn + MN + off) = s1;
            }
        }
    }
    __syncthreads();

    // ---- v = H^T y + rho D^T w (ops.jl:168), fed straight into the forward pass 0 ----
    float2* F0 = const_cast<float2*>(Xr);   // x is dead now
#pragma unroll
    for (int it = 0; it < NITF; ++it) {
        const int idx = tid + it * NT;
        if (idx < T * QF) {
            const int f = idx / QF, j = idx - f * QF;
            const float* w0a = W0 + f * M;
            const float* w0b = W0 + (f + 1) * M;
            const float* w1 = W1 + f * M;
            float2 v[RF];
#pragma unroll
            for (int r = 0; r < RF; ++r) {
                const int n = j + r * QF;
                const float2 a = *reinterpret_cast<const float2*>(w0a + 2 * n);
                const float2 b = *reinterpret_cast<const float2*>(w0b + 2 * n);
                const float2 c = *reinterpret_cast<const float2*>(w1 + 2 * n);
                const float cn = w1[(2 * n + 2) & (M - 1)];
                v[r].x = fmaf(rho, (a.x - b.x) + (c.x - c.y), preh[it][r].x);
                v[r].y = fmaf(rho, (a.y - b.y) + (c.y - cn), preh[it][r].y);
            }
            fly_core<L, RF, 0, false, 2>(v, j, tw);
            const int o = out_base<L, RF, 0>(j);
            if constexpr (P == 1) {
#pragma unroll
                for (int r = 0; r < RF; ++r) F0[f * L + o + r] = v[r];
            } else {
#pragma unroll
                for (int r = 0; r < RF; ++r) F0[f * L + o + r] = v[r];
            }
        }
    }
    __syncthreads();
    float2* Z;
    if constexpr (P == 1) {
        Z = F0;
    } else if constexpr (P == 2) {
        float2* Zb = reinterpret_cast<float2*>(W0);   // w0 dead now
        plan_pass<L, 1, true, false, 2>(T, tw, LdsIO{F0, L}, LdsIO{Zb, L});
        __syncthreads();
        Z = Zb;
    } else {
        float2* Zb = reinterpret_cast<float2*>(W0);
        plan_pass<L, 1, true, false, 2>(T, tw, LdsIO{F0, L}, LdsIO{Zb, L});
        __syncthreads();
        plan_pass<L, 2, true, false, 2>(T, tw, LdsIO{Zb, L}, LdsIO{Cf, L});
        __syncthreads();
        Z = Cf;
    }
    pack_store<L>(Z, spec0 + (size_t)plane * N * L, j0, T, N, tw);
}

template <int L, int T, int NT = kThreads>
__global__ __launch_bounds__(NT) void line_kernel(const float2* __restrict__ spec1, float2* __restrict__ spec0,
                                                  const float* __restrict__ s_old, float* __restrict__ s_new,
                                                  const float* __restrict__ hty, const float2* __restrict__ twM, int N,
                                                  const float* __restrict__ prm, int s_zero, Branches br = kOneSolve) {
    line_body<L, T, NT>(xcd_block(), spec1, spec0, s_old, s_new, hty, twM, N, prm, s_zero, br);
}

// ----------------------------------------------------------------------------------------------
// ISOTROPIC (block-thresholding) path, ops.jl:6,10.  pixelnorm sums s^2 over BOTH channels of EVERY
// plane of the batch, so the prox needs a batch-wide reduction between computing s and using it:
//   ISO_A  (per line tile, G planes per block): irFFT -> x -> s = Dx + u_old -> write s, and the
//          partial per-pixel sum of s0^2 + s1^2 over the block's G planes (no atomics)
//   ISO_R  (per pixel): n = sqrt(sum of partials); f = max(1 - tau/n, 0) with Julia's NaN
//          propagation (tau = 0 and n = 0 gives NaN, as the reference does)
//   ISO_B  (per line tile): z = f s, u = s - z, w = z - u -> v = H^T y + rho D^T w -> rFFT
// u_old for the next iteration is s - f s with the SAME f (kept in the workspace).
// ----------------------------------------------------------------------------------------------
__device__ __forceinline__ float max0_nan(float a) { return a != a ? a : fmaxf(a, 0.0f); }

template <int L, int T>
__global__ __launch_bounds__(kThreads) void iso_a_kernel(const float2* __restrict__ spec1,
                                                         const float* s_old, float* s_new,
                                                         const float* __restrict__ fmap, float* __restrict__ part,
                                                         const float2* __restrict__ twM, int N, int planes, int G,
                                                         int s_zero, int ngb = 0) {
    // planes: per branch; ngb: plane groups per branch (grid y = branches x ngb; 0: one branch).  Group g of branch
    // i sums planes i planes + g G ..; its partial map stays at its grid row, f at the branch's map
    constexpr int M = 2 * L;
    constexpr int M4 = M / 4;
    constexpr int TH = T + 1;           // one halo line on the left (x[j-1])
    constexpr int NE = T * M4;
    constexpr int NIT = (NE + kThreads - 1) / kThreads;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float2* tw = reinterpret_cast<float2*>(smem_raw);
    float2* X = tw + M;
    float2* Bf = X + TH * L;
    float2* Cf = Bf + TH * L;
    const XBlk xb = xcd_block();
    const int j0 = xb.x * T;
    const int grp = xb.y;
    const int nb_ = ngb > 0 ? ngb : (int)gridDim.y;
    const int bi = grp / nb_, gl = grp - bi * nb_;
    const size_t MN = (size_t)M * N;
    fmap += (size_t)bi * MN;
    const int tid = threadIdx.x;
    for (int t = tid; t < M; t += kThreads) tw[t] = twM[t];
    float4 acc[NIT], fo[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
        acc[it] = make_float4(0.f, 0.f, 0.f, 0.f);
        const int idx = tid + it * kThreads;
        const int t = idx / M4, i = (idx - t * M4) * 4;
        fo[it] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (!s_zero && idx < NE) fo[it] = *reinterpret_cast<const float4*>(fmap + (size_t)(j0 + t) * M + i);
    }
    const int p_end = bi * planes + min(planes, (gl + 1) * G);
    for (int plane = bi * planes + gl * G; plane < p_end; ++plane) {
        __syncthreads();   // previous plane's LDS readers are done
        load_lines<L>(spec1 + (size_t)plane * N * L, X, j0 - 1, TH, N);
        __syncthreads();
        auto uload = [&](int f, int n) { return unpack_z<L>(X + f * L, n, tw); };
        float2* Xr;
        if constexpr (Plan<L>::P == 1) {
            Xr = Bf;
            fpass<L, L, 0, true, 2>(TH, tw, uload, LdsIO{Bf, L});
        } else if constexpr (Plan<L>::P == 2) {
            Xr = X;
            fft_plan<L, false, true, 2>(TH, tw, Bf, Cf, L, uload, LdsIO{X, L});
        } else {
            Xr = Bf;
            plan_pass<L, 0, false, true, 2>(TH, tw, uload, LdsIO{Bf, L});
            __syncthreads();
            plan_pass<L, 1, false, true, 2>(TH, tw, LdsIO{Bf, L}, LdsIO{Cf, L});
            __syncthreads();
            plan_pass<L, 2, false, true, 2>(TH, tw, LdsIO{Cf, L}, LdsIO{Bf, L});
        }
        __syncthreads();
        const float* x = reinterpret_cast<const float*>(Xr);
        const float* so = s_old + (size_t)plane * 2 * MN;
        float* sn = s_new + (size_t)plane * 2 * MN;
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int idx = tid + it * kThreads;
            if (idx < NE) {
                const int t = idx / M4, i = (idx - t * M4) * 4;
                const size_t off = (size_t)(j0 + t) * M + i;
                const float4 xc = *reinterpret_cast<const float4*>(x + (t + 1) * M + i);
                const float4 xp = *reinterpret_cast<const float4*>(x + t * M + i);
                const float xl = x[(t + 1) * M + ((i - 1) & (M - 1))];
                float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0;
                if (!s_zero) {
                    a0 = *reinterpret_cast<const float4*>(so + off);
                    a1 = *reinterpret_cast<const float4*>(so + MN + off);
                }
                const float4 f = fo[it];
                // u_old = s_old - f s_old   (f from the previous iteration's batch norm)
                float4 s0, s1;
                s0.x = (xc.x - xp.x) + (a0.x - f.x * a0.x);
                s0.y = (xc.y - xp.y) + (a0.y - f.y * a0.y);
                s0.z = (xc.z - xp.z) + (a0.z - f.z * a0.z);
                s0.w = (xc.w - xp.w) + (a0.w - f.w * a0.w);
                s1.x = (xc.x - xl) + (a1.x - f.x * a1.x);
                s1.y = (xc.y - xc.x) + (a1.y - f.y * a1.y);
                s1.z = (xc.z - xc.y) + (a1.z - f.z * a1.z);
                s1.w = (xc.w - xc.z) + (a1.w - f.w * a1.w);
                *reinterpret_cast<float4*>(sn + off) = s0;
                *reinterpret_cast<float4*>(sn + MN + off) = s1;
                acc[it].x += s0.x * s0.x + s1.x * s1.x;
                acc[it].y += s0.y * s0.y + s1.y * s1.y;
                acc[it].z += s0.z * s0.z + s1.z * s1.z;
                acc[it].w += s0.w * s0.w + s1.w * s1.w;
            }
        }
    }
    float* pp = part + (size_t)grp * MN;
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
        const int idx = tid + it * kThreads;
        if (idx < NE) {
            const int t = idx / M4, i = (idx - t * M4) * 4;
            *reinterpret_cast<float4*>(pp + (size_t)(j0 + t) * M + i) = acc[it];
        }
    }
}

// nrm_out (optional) keeps the per-pixel batch norm for the adjoint (trajectory recording)
// Sum over the plane groups' maps at pixels base .. base+63: a block = 64 pixels x 4 group slices (slice
// s adds groups s, s+4, ...; 16 loads in flight per thread at 64 groups instead of 64 dependent ones),
// slices combined in a fixed order (deterministic).  The result is valid on slice 0 (threads 0..63).
__device__ __forceinline__ float group_sum(const float* __restrict__ part, int ngroups, size_t MN, size_t q,
                                           float* red) {
    const int slice = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float a = 0.0f;
    if (q < MN) {
#pragma unroll 4
        for (int g = slice; g < ngroups; g += 4) a += part[(size_t)g * MN + q];
    }
    red[threadIdx.x] = a;
    __syncthreads();
    float r = 0.0f;
    if (slice == 0) r = ((red[lane] + red[64 + lane]) + red[128 + lane]) + red[192 + lane];
    __syncthreads();
    return r;
}

// grid (blocks, branches): branch blockIdx.y sums its own ngroups partials (iso_a's groups of that branch)
__global__ __launch_bounds__(kThreads) void iso_r_kernel(const float* __restrict__ part, float* __restrict__ fmap,
                                                         int ngroups, size_t MN, const float* __restrict__ prm, float* __restrict__ nrm_out,
                                                         unsigned prm_f = 0) {
    const size_t bi = blockIdx.y;
    part += bi * ngroups * MN;
    fmap += bi * MN;
    if (nrm_out) nrm_out += bi * MN;
    const float tau = prm[bi * prm_f];   // device-resident scalars (setup_kernel)
    __shared__ float red[kThreads];
    for (size_t base = (size_t)blockIdx.x * 64; base < MN; base += (size_t)gridDim.x * 64) {
        const size_t q = base + (threadIdx.x & 63);
        const float acc = group_sum(part, ngroups, MN, q, red);
        if (threadIdx.x < 64 && q < MN) {
            const float nrm = sqrtf(acc);
            fmap[q] = max0_nan(1.0f - tau / nrm);   // BT factor, ops.jl:10
            if (nrm_out) nrm_out[q] = nrm;
        }
    }
}

// sharded batch (admm_batch_reducer): ISO_R splits into the per-shard sum, the caller's cross-shard
// all-reduce of that M x N map, and the BT factor
__global__ __launch_bounds__(kThreads) void iso_sum_kernel(const float* __restrict__ part, float* __restrict__ acc,
                                                           int ngroups, size_t MN) {
    __shared__ float red[kThreads];
    for (size_t base = (size_t)blockIdx.x * 64; base < MN; base += (size_t)gridDim.x * 64) {
        const size_t q = base + (threadIdx.x & 63);
        const float a = group_sum(part, ngroups, MN, q, red);
        if (threadIdx.x < 64 && q < MN) acc[q] = a;
    }
}

__global__ __launch_bounds__(kThreads) void iso_fin_kernel(float* __restrict__ fmap, size_t MN, const float* __restrict__ prm,
                                                           float* __restrict__ nrm_out) {
    const float tau = prm[0];   // device-resident scalars (setup_kernel)
    for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < MN; q += (size_t)gridDim.x * blockDim.x) {
        const float nrm = sqrtf(fmap[q]);   // fmap holds the all-reduced sum of squares
        fmap[q] = max0_nan(1.0f - tau / nrm);
        if (nrm_out) nrm_out[q] = nrm;
    }
}

template <int L, int T>
__global__ __launch_bounds__(kThreads) void iso_b_kernel(const float* __restrict__ s_new, const float* __restrict__ fmap,
                                                         const float* __restrict__ hty, float2* __restrict__ spec0,
                                                         const float2* __restrict__ twM, int N, const float* __restrict__ prm,
                                                         Branches br = kOneSolve) {
    constexpr int M = 2 * L;
    constexpr int M4 = M / 4;
    constexpr int P = Plan<L>::P;
    constexpr int RF = plan_radix<L, 0, true>();
    constexpr int QF = L / RF;
    constexpr int NE = (T + 1) * M4;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float2* tw = reinterpret_cast<float2*>(smem_raw);
    float* W0 = reinterpret_cast<float*>(tw + M);   // T+1 lines
    float* W1 = W0 + (T + 1) * M;                   // T lines
    float2* F0 = reinterpret_cast<float2*>(W1 + T * M);   // T lines
    float2* F1 = F0 + T * L;                               // T lines
    const XBlk xb = xcd_block();
    const int plane = xb.y;
    const int j0 = xb.x * T;
    const size_t MN = (size_t)M * N;
    const int tid = threadIdx.x;
    const BranchOf bo = branch_of(br, plane);
    fmap += (size_t)bo.i * MN;
    const float rho = prm[(size_t)bo.i * br.prm_f + 1];   // device-resident scalars (setup_kernel)
    const float* sp = s_new + (size_t)plane * 2 * MN;
    const float* hp = hty ? hty + bo.in_plane * MN : nullptr;   // NULL: H^T y enters spectrally (YH_ADD)
    for (int t = tid; t < M; t += kThreads) tw[t] = twM[t];
    for (int idx = tid; idx < NE; idx += kThreads) {
        const int t = idx / M4, i = (idx - t * M4) * 4;
        const size_t off = (size_t)((j0 + t) & (N - 1)) * M + i;
        const float4 f = *reinterpret_cast<const float4*>(fmap + off);
        const float4 a = *reinterpret_cast<const float4*>(sp + off);
        float4 w;
        // z = f s ; u = s - z ; w = z - u
        w.x = f.x * a.x - (a.x - f.x * a.x);
        w.y = f.y * a.y - (a.y - f.y * a.y);
        w.z = f.z * a.z - (a.z - f.z * a.z);
        w.w = f.w * a.w - (a.w - f.w * a.w);
        *reinterpret_cast<float4*>(W0 + t * M + i) = w;
        if (t < T) {
            const float4 b = *reinterpret_cast<const float4*>(sp + MN + off);
            w.x = f.x * b.x - (b.x - f.x * b.x);
            w.y = f.y * b.y - (b.y - f.y * b.y);
            w.z = f.z * b.z - (b.z - f.z * b.z);
            w.w = f.w * b.w - (b.w - f.w * b.w);
            *reinterpret_cast<float4*>(W1 + t * M + i) = w;
        }
    }
    __syncthreads();
    for (int idx = tid; idx < T * QF; idx += kThreads) {
        const int f = idx / QF, j = idx - f * QF;
        const float2* hl = hp ? reinterpret_cast<const float2*>(hp + (size_t)(j0 + f) * M) : nullptr;
        float2 v[RF];
#pragma unroll
        for (int r = 0; r < RF; ++r) {
            const int n = j + r * QF;
            const float2 hv = hl ? hl[n] : make_float2(0.f, 0.f);
            const float2 a = *reinterpret_cast<const float2*>(W0 + f * M + 2 * n);
            const float2 b = *reinterpret_cast<const float2*>(W0 + (f + 1) * M + 2 * n);
            const float2 c = *reinterpret_cast<const float2*>(W1 + f * M + 2 * n);
            const float cn = W1[f * M + ((2 * n + 2) & (M - 1))];
            v[r].x = fmaf(rho, (a.x - b.x) + (c.x - c.y), hv.x);
            v[r].y = fmaf(rho, (a.y - b.y) + (c.y - cn), hv.y);
        }
        fly_core<L, RF, 0, false, 2>(v, j, tw);
        const int o = out_base<L, RF, 0>(j);
#pragma unroll
        for (int r = 0; r < RF; ++r) F0[f * L + o + r] = v[r];
    }
    __syncthreads();
    float2* Z;
    if constexpr (P == 1) {
        Z = F0;
    } else if constexpr (P == 2) {
        plan_pass<L, 1, true, false, 2>(T, tw, LdsIO{F0, L}, LdsIO{F1, L});
        __syncthreads();
        Z = F1;
    } else {
        plan_pass<L, 1, true, false, 2>(T, tw, LdsIO{F0, L}, LdsIO{F1, L});
        __syncthreads();
        plan_pass<L, 2, true, false, 2>(T, tw, LdsIO{F1, L}, LdsIO{F0, L});
        __syncthreads();
        Z = F0;
    }
    pack_store<L>(Z, spec0 + (size_t)plane * N * L, j0, T, N, tw);
}

// y_bar of a multi-branch solve: out[j] = sum over the nbr branches of v[i * n + j], branch order fixed
// (deterministic).  v: nbr consecutive blocks of n floats (each branch's input gradient).
__global__ __launch_bounds__(kThreads) void branch_sum_kernel(const float* __restrict__ v, float* __restrict__ out,
                                                              size_t n, int nbr) {
    for (size_t j = (size_t)blockIdx.x * kThreads + threadIdx.x; j < n; j += (size_t)gridDim.x * kThreads) {
        float a = v[j];
        for (int i = 1; i < nbr; ++i) a += v[(size_t)i * n + j];
        out[j] = a;
    }
}

}  // namespace admm
