// plane_launch.hip -- translation unit of the fused per-plane kernel (built without packed FP32,
// see plane_api.hpp) and its host launchers.
#include "plane_api.hpp"
#include "plane_kernel.hip"
#include "plane_iso.hip"

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

static Branches one_branch() { return Branches{1, 1, 1, 0u, 0u}; }

template <bool PSF, int TRAJ>
static void launch_one(const float* y, float* x_out, const Tables& t, float2* hln, float4* sln, const float* prm,
                       int K, size_t planes, hipStream_t s, float4* traj, const Branches& br,
                       unsigned* masks) {
    (void)hipFuncSetAttribute((const void*)plane256_kernel<PSF, 0, TRAJ>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kLdsBytes);
    hipLaunchKernelGGL((plane256_kernel<PSF, 0, TRAJ>), dim3((unsigned)planes), dim3(kPT), kLdsBytes, s, y, x_out,
                       t.Cf, t.C0b, t.Gf, t.G0b, hln, sln, prm, K, nullptr, traj,
                       planes * 64 * kPT, br, masks, planes * 16 * kPT);
}

hipError_t launch_plane(const float* y, float* x_out, const void* tables, bool psf, float2* hln, float4* sln,
                        const float* prm, int K, size_t planes, hipStream_t s, float4* traj,
                        const Branches* brp, unsigned* masks) {
    const Tables t = carve(tables);
    const Branches br = brp ? *brp : one_branch();
    const int mode = traj ? 1 : masks ? 2 : 0;
#define X(P, M)                                                                                     \
    if (psf == P && mode == M) {                                                                    \
        launch_one<P, M>(y, x_out, t, hln, sln, prm, K, planes, s, traj, br, masks);               \
        return hipGetLastError();                                                                   \
    }
    X(false, 0) X(false, 1) X(false, 2) X(true, 0) X(true, 1) X(true, 2)
#undef X
    return hipErrorInvalidValue;
}


hipError_t launch_dx_lane(const float* xK, float4* dxK, size_t planes, hipStream_t s, const Branches* brp) {
    hipLaunchKernelGGL(dx_lane_kernel, dim3(64 * kPT / 256, (unsigned)planes), dim3(256), 0, s, xK, dxK,
                       brp ? *brp : one_branch());
    return hipGetLastError();
}

hipError_t launch_plane_adj(const float* xbar, const void* tables, const void* traj, const float4* dxK, float4* sbar,
                            float2* vsl, float* vout, double* part, const float* prm, int K, size_t planes,
                            hipStream_t s, const Branches* brp, bool masks) {
    const Tables t = carve(tables);
    const Branches br = brp ? *brp : one_branch();
    if (masks && dxK) return hipErrorInvalidValue;   // rho_bar needs the full trajectory
    const size_t slot = masks ? planes * 16 * kPT : planes * 64 * kPT;
#define X(MK, WV)                                                                                              \
    if (masks == MK && (vout != nullptr) == WV) {                                                             \
        (void)hipFuncSetAttribute((const void*)plane256_adj_kernel<MK, WV>,                                   \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBytes);                \
        hipLaunchKernelGGL((plane256_adj_kernel<MK, WV>), dim3((unsigned)planes), dim3(kPT), kLdsBytes, s,    \
                           xbar, t.Cf, t.C0b, traj, slot, dxK, sbar, vsl, vout, part, prm, K, br);                 \
    }
    X(false, false) X(false, true) X(true, false) X(true, true)
#undef X
    return hipGetLastError();
}

hipError_t launch_plane_iso(const float* y, float* x_out, const void* tables, bool psf, float2* hln, const float4* s_in,
                            float4* s_out, const float2* fmap, float2* qpart, const float* prm, int k, int K,
                            size_t planes, hipStream_t s, const Branches* brp) {
    const Tables t = carve(tables);
    const Branches br = brp ? *brp : one_branch();
    if (psf) {
        (void)hipFuncSetAttribute((const void*)plane256_iso_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)kLdsBytes);
        hipLaunchKernelGGL(plane256_iso_kernel<true>, dim3((unsigned)planes), dim3(kPT), kLdsBytes, s, y, x_out, t.Cf,
                           t.C0b, t.Gf, t.G0b, hln, s_in, s_out, fmap, qpart, prm, k, K, br);
    } else {
        (void)hipFuncSetAttribute((const void*)plane256_iso_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)kLdsBytes);
        hipLaunchKernelGGL(plane256_iso_kernel<false>, dim3((unsigned)planes), dim3(kPT), kLdsBytes, s, y, x_out, t.Cf,
                           t.C0b, t.Gf, t.G0b, hln, s_in, s_out, fmap, qpart, prm, k, K, br);
    }
    return hipGetLastError();
}

hipError_t launch_iso_norm(const float2* qpart, float2* fmap, float2* nrm, const float* prm, size_t planes,
                           hipStream_t s, const Branches* brp, float2* sum_out, const float2* sum_in) {
    const Branches br = brp ? *brp : Branches{(int)planes, 1, 1, 0u, 0u};
    hipLaunchKernelGGL(iso_norm_kernel, dim3(64 * kPT / 64, (unsigned)br.nbr), dim3(256), 0, s, qpart, fmap, nrm, prm, br,
                       sum_out, sum_in);
    return hipGetLastError();
}

hipError_t launch_plane_isoadj(const float* xbar, const void* tables, const float4* traj, size_t tslot, const float2* nrm,
                               size_t nslot, float2* vbuf, float4* sbar, const float2* Rmap, float2* rpart, float2* vsl,
                               float* vout, const float* prm, int k, int K, size_t planes, hipStream_t s,
                               const Branches* brp) {
    const Tables t = carve(tables);
    const Branches br = brp ? *brp : one_branch();
    if (vout) {
        (void)hipFuncSetAttribute((const void*)plane256_isoadj_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)kLdsBytes);
        hipLaunchKernelGGL(plane256_isoadj_kernel<true>, dim3((unsigned)planes), dim3(kPT), kLdsBytes, s, xbar, t.Cf,
                           t.C0b, traj, tslot, nrm, nslot, vbuf, sbar, Rmap, rpart, vsl, vout, prm, k, K, br);
    } else {
        (void)hipFuncSetAttribute((const void*)plane256_isoadj_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)kLdsBytes);
        hipLaunchKernelGGL(plane256_isoadj_kernel<false>, dim3((unsigned)planes), dim3(kPT), kLdsBytes, s, xbar, t.Cf,
                           t.C0b, traj, tslot, nrm, nslot, vbuf, sbar, Rmap, rpart, vsl, vout, prm, k, K, br);
    }
    return hipGetLastError();
}

hipError_t launch_iso_radj(const float2* rpart, float2* Rmap, const float2* nrm1, double* part, size_t part_branch,
                           const float* prm, size_t planes, hipStream_t s, const Branches* brp) {
    const Branches br = brp ? *brp : Branches{(int)planes, 1, 1, 0u, 0u};
    hipLaunchKernelGGL(iso_radj_kernel, dim3(64 * kPT / 64, (unsigned)br.nbr), dim3(256), 0, s, rpart, Rmap, nrm1, part,
                       part_branch, prm, br);
    return hipGetLastError();
}

}  // namespace plane
}  // namespace admm
