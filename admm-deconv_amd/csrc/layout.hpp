// layout.hpp -- how one call carves the caller's workspace (host only).  Shared by admm_capi.hip (the
// library) and devtest.hip (tests read a recording's trajectory back through these offsets).
#pragma once
#include <cstddef>

#include "plane_api.hpp"

namespace admm {
namespace layout {

inline bool is_pow2(int n) { return n > 0 && (n & (n - 1)) == 0; }
// The tuned kernels cover power-of-two 4 <= M <= 1024, 2 <= N <= 1024; every other shape from 2 x 2 up
// to 4096 x 4096 runs the runtime-length path (admm_generic.hip).
inline bool pow2_shape(int M, int N) { return is_pow2(M) && is_pow2(N) && M >= 4 && M <= 1024 && N >= 2 && N <= 1024; }
inline bool generic_shape(int M, int N) { return !pow2_shape(M, N); }
// The fused per-plane kernel (plane_kernel.hip) covers 256 x 256 planes with the anisotropic prox.
inline bool fused_shape(int M, int N, bool iso) { return M == 256 && N == 256 && !iso; }
// The isotropic split-iteration kernels (plane_iso.hip) cover 256 x 256 as well; both need the lane-native tables.
inline bool fused_tables_shape(int M, int N) { return M == 256 && N == 256; }
inline size_t align_up(size_t v) { return (v + 255) & ~size_t(255); }

// Planes per isotropic plane-group block (ISO_A / ISO_ADJ_A keep a group's partial batch sums in
// registers; ISO_R / ISO_ADJ_R add the groups' maps).  At most 64 groups: enough blocks to fill the chip
// (64 x N/T), while the group maps stay small (64 x M x N floats).  16 planes per group for every batch
// left the c5 batch (192 planes) at 12 x 32 = 384 blocks, a block and a half per CU.
inline int iso_group(size_t planes) { return (int)((planes + 63) / 64); }
inline int iso_ngroups(size_t planes) {
    const int g = iso_group(planes);
    return (int)((planes + g - 1) / g);
}

struct Layout {
    size_t prm, twM, twN, C, G, hty, sA, sB, spec0, spec1, fmap, part, F, xg, total;
};

// Forward workspace (256-B aligned carve-outs); see DESIGN.md s3.
inline Layout make_layout(int M, int N, size_t planes, bool psf, bool iso) {
    Layout L{};
    size_t off = 0;
    auto take = [&](size_t bytes) {
        size_t o = off;
        off = align_up(off + bytes);
        return o;
    };
    const size_t MN = (size_t)M * N;
    L.prm = take(16);   // {tau, rho, lambda} resolved on the device (setup_kernel)
    L.twM = take((size_t)M * 8);
    L.twN = take((size_t)N * 8);
    L.C = take((size_t)(M / 2 + 1) * N * 4);
    L.G = psf ? take((size_t)(M / 2 + 1) * N * 8) : 0;
    // H^T y (CU-resident and fused paths, PSF only) -- or, on the 2-pass and runtime-length paths, Y_h = F(H^T y) as
    // the column pass's 2-D spectrum (packed M/2 x N, or M/2+1 x N bins on the generic path), with or without a PSF
    L.hty = take(planes * (generic_shape(M, N) ? (size_t)(M / 2 + 1) * N * 8 : MN * 4));
    L.sA = take(planes * 2 * MN * 4);
    L.sB = take(planes * 2 * MN * 4);
    // N lines x M/2 complex (packed) -- or M/2 + 1 bins per line on the generic path
    const size_t spec_bytes = generic_shape(M, N) ? planes * (size_t)(M / 2 + 1) * N * 8 : planes * MN * 4;
    // the fused 256^2 kernels keep their lane-native H^T y in spec0, at a skewed plane stride
    L.spec0 = take(fused_tables_shape(M, N) && admm::plane::hty_bytes(planes) > spec_bytes ? admm::plane::hty_bytes(planes)
                                                                                            : spec_bytes);
    L.spec1 = take(spec_bytes);
    L.xg = generic_shape(M, N) ? take(planes * MN * 4) : 0;
    L.fmap = iso ? take(MN * 4) : 0;
    L.part = iso ? take((size_t)iso_ngroups(planes) * MN * 4) : 0;
    L.F = fused_tables_shape(M, N) ? take(admm::plane::tables_bytes()) : 0;
    L.total = off;
    return L;
}

// Head of the backward workspace: the forward layout, then the recorded trajectory and the reverse
// sweep's state.  `end` is where the rest of the backward layout (admm_capi.hip make_bwd_layout) starts.
struct BwdHead {
    Layout f;
    size_t traj_s;   // (K-1) x planes x 2 x M x N floats: s_k, k = 1..K-1 (natural or lane-native layout)
    size_t traj_v, sig, sbA, sbB, vsum;
    size_t traj_n;   // isotropic only: (K-1) x M x N batch norms |s_k|
    size_t end;
};

// masks: the trajectory holds the fused kernel's ST mask bytes (ADMM_REC_MASKS), 32 KiB per plane and
// iteration, instead of s_k (512 KiB)
inline BwdHead bwd_head(int M, int N, size_t planes, int kh, int maxit, bool want_h, bool iso, bool masks = false) {
    BwdHead b{};
    b.f = make_layout(M, N, planes, kh > 0, iso);
    size_t off = b.f.total;
    auto take = [&](size_t bytes) {
        size_t o = off;
        off = align_up(off + bytes);
        return o;
    };
    const size_t MN = (size_t)M * N;
    const int K = maxit < 1 ? 1 : maxit;
    const bool gen = generic_shape(M, N);
    const bool hq = want_h && kh > 0;
    b.traj_s = take((size_t)(K > 1 ? K - 1 : 1) * planes * (masks ? MN / 2 : 2 * MN * 4));
    // forward dim-2 spectra per iteration: packed M/2 x N (power of two) or M/2+1 x N bins (generic)
    b.traj_v = hq ? take((size_t)K * planes * (gen ? (size_t)(M / 2 + 1) * N * 8 : MN * 4)) : 0;
    b.sig = hq ? take((size_t)(M / 2 + 1) * N * 16) : 0;
    b.sbA = take(planes * 2 * MN * 4);
    b.sbB = take(planes * 2 * MN * 4);
    b.vsum = take(planes * MN * 4);
    b.traj_n = iso ? take((size_t)(K > 1 ? K - 1 : 1) * MN * 4) : 0;
    b.end = off;
    return b;
}

}  // namespace layout
}  // namespace admm
