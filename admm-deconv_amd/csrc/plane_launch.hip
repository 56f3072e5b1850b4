// plane_launch.hip -- translation unit of the fused per-plane kernel (built without packed FP32,
// see plane_api.hpp) and its host launchers.
#include "plane_api.hpp"
#include "plane_kernel.hip"

namespace admm {
namespace plane {

static_assert(kTab == kTabEntries, "table size");

namespace {
struct Tables {
    float* Cf;
    float* C0b;
    float2* Gf;
    float2* G0b;
};
Tables carve(const void* base) {
    float* Cf = static_cast<float*>(const_cast<void*>(base));
    float* C0b = Cf + kTab;
    float2* Gf = reinterpret_cast<float2*>(C0b + 256);
    float2* G0b = Gf + kTab;
    return {Cf, C0b, Gf, G0b};
}
}  // namespace

hipError_t launch_tables(const float* Ct, const float2* Gt, void* tables, hipStream_t s) {
    const Tables t = carve(tables);
    hipLaunchKernelGGL(tables_kernel, dim3(kTab / 256), dim3(256), 0, s, Ct, Gt, t.Cf, t.C0b, t.Gf, t.G0b);
    return hipGetLastError();
}

template <bool PSF, bool TRAJ>
static void launch_one(const float* y, float* x_out, const Tables& t, float2* hln, float4* sln, const float* prm,
                       int K, size_t planes, hipStream_t s, int stagger, float4* traj) {
    (void)hipFuncSetAttribute((const void*)plane256_kernel<PSF, 0, TRAJ>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kLdsBytes);
    hipLaunchKernelGGL((plane256_kernel<PSF, 0, TRAJ>), dim3((unsigned)planes), dim3(kPT), kLdsBytes, s, y, x_out,
                       t.Cf, t.C0b, t.Gf, t.G0b, hln, sln, prm, K, nullptr, stagger, traj,
                       planes * 64 * kPT);
}

hipError_t launch_plane(const float* y, float* x_out, const void* tables, bool psf, float2* hln, float4* sln,
                        const float* prm, int K, size_t planes, hipStream_t s, float4* traj, int stagger) {
    const Tables t = carve(tables);
    if (psf) {
        if (traj) launch_one<true, true>(y, x_out, t, hln, sln, prm, K, planes, s, stagger, traj);
        else launch_one<true, false>(y, x_out, t, hln, sln, prm, K, planes, s, stagger, traj);
    } else {
        if (traj) launch_one<false, true>(y, x_out, t, hln, sln, prm, K, planes, s, stagger, traj);
        else launch_one<false, false>(y, x_out, t, hln, sln, prm, K, planes, s, stagger, traj);
    }
    return hipGetLastError();
}


hipError_t launch_dx_lane(const float* xK, float4* dxK, size_t planes, hipStream_t s) {
    hipLaunchKernelGGL(dx_lane_kernel, dim3(64 * kPT / 256, (unsigned)planes), dim3(256), 0, s, xK, dxK);
    return hipGetLastError();
}

hipError_t launch_plane_adj(const float* xbar, const void* tables, const float4* traj, const float4* dxK, float4* sbar,
                            float2* vsl, float* vout, double* part, const float* prm, int K, size_t planes,
                            hipStream_t s) {
    const Tables t = carve(tables);
    (void)hipFuncSetAttribute((const void*)plane256_adj_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kLdsBytes);
    hipLaunchKernelGGL(plane256_adj_kernel, dim3((unsigned)planes), dim3(kPT), kLdsBytes, s, xbar, t.Cf, t.C0b, traj,
                       planes * 64 * kPT, dxK, sbar, vsl, vout, part, prm, K);
    return hipGetLastError();
}

}  // namespace plane
}  // namespace admm
