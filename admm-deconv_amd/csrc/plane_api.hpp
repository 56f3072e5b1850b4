// plane_api.hpp -- host interface of the fused per-plane kernel (plane_launch.hip).
//
// The fused kernel lives in its own translation unit because it is compiled WITHOUT packed-FP32
// VALU ops (-Xclang -target-feature -Xclang -packed-fp32-ops): with ROCm 7.2's gfx950 codegen the
// register-dense code of this kernel produced nondeterministic lane corruption in v_pk_*_f32 results
// (lanes 10-15 of a 16-lane group, found with a per-phase state dump).  Without
// packed FP32 the kernel is bitwise deterministic.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

namespace admm {
namespace plane {

constexpr int kPlaneM = 256, kPlaneN = 256;

// Several independent solves in one grid: the branches of a Flux Parallel(chcat, ...) that share their
// input (the denoiser, src/nets/net_build.jl:113-125).  Grid plane q is plane q % ppb of the shared input,
// solved with branch i = q / ppb's tables and scalars; its output goes to the chcat position of branch i
// (image b, channel i * P + p of a (B, nbr * P, N, M) tensor).  A single solve is nbr = 1.
struct Branches {
    int ppb;          // planes per branch (B * P)
    int nbr;          // branches
    int P;            // channels per image of one branch
    unsigned tab_f;   // floats between the branches' lane-native table blocks (tables_bytes() / 4)
    unsigned prm_f;   // floats between the branches' {tau, rho, lambda} blocks
};
// Where grid plane q reads and writes (above).  The 2-pass kernels (admm_kernels.hip) take the same struct, with
// tab_f = floats between the branches' 2-pass C tables.
struct BranchOf {
    int i;
    size_t in_plane, out_plane;
};
__host__ __device__ inline BranchOf branch_of(const Branches& br, size_t plane) {
    if (br.nbr == 1) return {0, plane, plane};
    const int i = (int)(plane / (size_t)br.ppb);
    const size_t loc = plane - (size_t)i * br.ppb;
    const size_t b = loc / (size_t)br.P, p = loc - b * br.P;
    return {i, loc, (b * br.nbr + i) * br.P + p};
}
constexpr int kTabEntries = 2 * 32 * 512;   // lane-native spectral table entries (= 256 x 128)

// bytes of the lane-native tables (Cf, C0b, Gf, G0b) carved from the workspace
inline size_t tables_bytes() { return (size_t)kTabEntries * 12 + 256 * 12 + 256; }
// Plane stride of the lane-native H^T y (float2 units): 256 KiB + 1 KiB.  At a power-of-two stride every
// workgroup's row phase, in lock-step with the others, reads H^T y at the same offset of its own plane; the
// 1 KiB skew spreads those reads over the memory channels: c2 164k -> 168-170k, c3's 256-plane shard
// 149-151k -> 157-158k img/s (profiles/r06_plane_pad_ab*.jsonl; the s state's stride showed no such effect).
constexpr size_t kHtyStrideF2 = 64 * 512 + 128;
inline size_t hty_bytes(size_t planes) { return planes * kHtyStrideF2 * 8; }

// Cf/C0b/Gf/G0b from the 2-pass tables Ct/Gt (Gt may be NULL: no PSF)
hipError_t launch_tables(const float* Ct, const float2* Gt, void* tables, hipStream_t s);

// all K >= 1 iterations for `planes` planes of 256 x 256; hln: planes x 256 KiB, sln: planes x 512 KiB
// traj != NULL: record s_1..s_{K-1} for the adjoint, slot k-1 at traj + (k-1) * planes * 64 * 512
// (lane-native: float4 (s0[p], s0[p+1], s1[p], s1[p+1]) of pixel pair p = 4n + 2h of line r at
// [plane][n][2r + h]; s0 = x - x(line r-1), s1 = x - x(pixel p-1)); sln is then unused
// prm: device {tau, rho, lambda} (setup_kernel)
// masks != NULL (and traj NULL): record only the ST mask bits of s_1..s_{K-1} (plane_kernel.hip mask_byte),
// slot k-1 at masks + (k-1) * planes * 16 * 512 dwords, for a reverse sweep without rho_bar.
// br (NULL = one solve): several branches in one grid; tables / prm then hold br->nbr consecutive blocks.
hipError_t launch_plane(const float* y, float* x_out, const void* tables, bool psf, float2* hln, float4* sln,
                        const float* prm, int K, size_t planes, hipStream_t s, float4* traj = nullptr,
                        const Branches* br = nullptr, unsigned* masks = nullptr);


// Reverse sweep of the anisotropic solve on the fused trajectory (plane256_adj_kernel):
// launch_dx_lane writes D x_K (x_K = the forward output, natural layout) in the lane-native s layout;
// launch_plane_adj runs steps K..1 for every plane.  traj: the forward's s_1..s_{K-1}; sbar, vsl: planes x
// 512 KiB / 256 KiB of state; vout: Vsum = sum_k vbar_k (natural layout; = y_bar without a PSF);
// part: 2 doubles per plane (rho_bar, tau_bar partial sums, fixed summation order).
hipError_t launch_dx_lane(const float* xK, float4* dxK, size_t planes, hipStream_t s, const Branches* br = nullptr);
// masks: traj is the mask-bit trajectory (dxK must be NULL: no rho_bar).  br: as in launch_plane (x_bar in the
// chcat layout; vout and part per grid plane).
hipError_t launch_plane_adj(const float* xbar, const void* tables, const void* traj, const float4* dxK, float4* sbar,
                            float2* vsl, float* vout, double* part, const float* prm, int K, size_t planes,
                            hipStream_t s, const Branches* br = nullptr, bool masks = false);

// Isotropic (BT) solve at 256 x 256 (plane_iso.hip): iteration k = 0 .. K-1 of every plane (hln: H^T y,
// lane-native, written at k = 0; s_in / s_out: s_k / s_{k+1}, the same state buffer, or trajectory slots k-1 / k
// when recording; fmap: the branch's lane-native BT factor f_k, k > 0; qpart: per plane |s_{k+1}|^2 partials),
// then, between iterations, launch_iso_norm (f_{k+1} and, when nrm is given, |s_{k+1}|, per branch from qpart;
// a sharded batch: sum_out = this shard's sums only, then, after the caller's all-reduce, sum_in = the sums).
// One plane's maps are 64 x 512 float2.
hipError_t launch_plane_iso(const float* y, float* x_out, const void* tables, bool psf, float2* hln, const float4* s_in,
                            float4* s_out, const float2* fmap, float2* qpart, const float* prm, int k, int K,
                            size_t planes, hipStream_t s, const Branches* br = nullptr);
hipError_t launch_iso_norm(const float2* qpart, float2* fmap, float2* nrm, const float* prm, size_t planes,
                           hipStream_t s, const Branches* br = nullptr, float2* sum_out = nullptr,
                           const float2* sum_in = nullptr);
// Reverse step k = K .. 1 of the isotropic solve on that recording (traj: s_1..s_{K-1}, slot stride tslot
// float4; nrm: |s_1|..|s_{K-1}|, slot stride nslot float2), no rho_bar; vbuf / sbar / Rmap / rpart / vsl:
// lane-native vbar_k, sbar_k, R map (per branch), R partials (per plane), Vsum; vout: Vsum in the natural
// layout (NULL: not wanted).  Then (k >= 2) launch_iso_radj: R_k and this step's tau_bar partial rows
// (part: 512 rows of (0, tau_bar) per branch, branch stride part_branch doubles).
hipError_t launch_plane_isoadj(const float* xbar, const void* tables, const float4* traj, size_t tslot, const float2* nrm,
                               size_t nslot, float2* vbuf, float4* sbar, const float2* Rmap, float2* rpart, float2* vsl,
                               float* vout, const float* prm, int k, int K, size_t planes, hipStream_t s,
                               const Branches* br = nullptr);
hipError_t launch_iso_radj(const float2* rpart, float2* Rmap, const float2* nrm1, double* part, size_t part_branch,
                           const float* prm, size_t planes, hipStream_t s, const Branches* br = nullptr);

}  // namespace plane
}  // namespace admm
