// admm_launch.hip -- launch sequencing of the ADMM solve (see capi_internal.hpp): the 2-pass kernels
//   SETUP  (twiddles + C, ops.jl:22-37)
//   PREP   (H^T y once + first line rFFT, ops.jl:71-81 / :168 first iteration)
//   K x COLUMN, (K-1) x LINE, 1 x FINAL                (ops.jl:166-174)
// and the fused / CU-resident / runtime-length paths and reverse sweeps, enqueued on the caller's stream
// exactly as plan_paths (admm_paths.hip) decided.  Reference: /root/reference/src/ops/ops.jl:99-188.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "capi_internal.hpp"
#include "admm_kernels.hip"
#include "admm_generic.hip"
#include "admm_backward.hip"
#include "admm_generic_bwd.hip"
#include "smooth_api.hpp"
#include "resident_api.hpp"

namespace admm_capi {

using namespace admm;

// ---- template dispatch -----------------------------------------------------------------------
using namespace admm;

template <typename K>
void set_lds(K kernel, size_t lds) {
    if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

// (L, T) pairs that line_T() can return
#define ADMM_LT_CASES(X)                                                                           \
    X(2, 2) X(2, 4) X(2, 8) X(2, 16) X(4, 2) X(4, 4) X(4, 8) X(4, 16) X(8, 2) X(8, 4) X(8, 8) X(8, 16) \
    X(16, 2) X(16, 4) X(16, 8) X(16, 16) X(32, 2) X(32, 4) X(32, 8) X(32, 16) X(64, 2) X(64, 4)      \
    X(64, 8) X(64, 16) X(128, 2) X(128, 4) X(128, 8) X(128, 16) X(256, 2) X(256, 4) X(256, 8)       \
    X(512, 2) X(512, 4)
#define ADMM_N_CASES(X) X(2) X(4) X(8) X(16) X(32) X(64) X(128) X(256) X(512) X(1024)

// br / map (several branches in one grid): the line transforms read / write the shared input plane or the chcat
// plane of each grid plane (admm_kernels.hip PlaneMap)
int launch_line_fwd(int L, int T, dim3 g, size_t lds, hipStream_t s, const float* src, float2* spec,
                    const float2* twM, int N, const Branches& br = kOneSolve, int map = kMapGrid) {
#define X(l, t)                                                                     \
    if (L == l && T == t) {                                                         \
        set_lds(line_fwd_kernel<l, t>, lds);                                        \
        line_fwd_kernel<l, t><<<g, kThreads, lds, s>>>(src, spec, twM, N, br, map); \
        return 0;                                                                   \
    }
    ADMM_LT_CASES(X)
#undef X
    return -1;
}

int launch_line_inv(int L, int T, dim3 g, size_t lds, hipStream_t s, const float2* spec, float* dst,
                    const float2* twM, int N, const Branches& br = kOneSolve, int map = kMapGrid) {
#define X(l, t)                                                                     \
    if (L == l && T == t) {                                                         \
        set_lds(line_inv_kernel<l, t>, lds);                                        \
        line_inv_kernel<l, t><<<g, kThreads, lds, s>>>(spec, dst, twM, N, br, map); \
        return 0;                                                                   \
    }
    ADMM_LT_CASES(X)
#undef X
    return -1;
}

int launch_line(int L, int T, dim3 g, size_t lds, hipStream_t s, const float2* spec1, float2* spec0,
                const float* so, float* sn, const float* hty, const float2* twM, int N, const float* prm,
                int sz, int nt = kThreads, const Branches& br = kOneSolve) {
    if (nt != kThreads) {   // wider blocks at 512-point lines (update kernel, line_T_upd)
#define X(l, t, n)                                                                                       \
        if (L == l && T == t && nt == n) {                                                               \
            set_lds(line_kernel<l, t, n>, lds);                                                          \
            line_kernel<l, t, n><<<g, n, lds, s>>>(spec1, spec0, so, sn, hty, twM, N, prm, sz, br);     \
            return 0;                                                                                    \
        }
        X(256, 8, 512) X(256, 16, 1024) X(256, 4, 512) X(256, 8, 1024)
#undef X
        return -1;
    }
#define X(l, t)                                                                                          \
    if (L == l && T == t) {                                                                              \
        set_lds(line_kernel<l, t>, lds);                                                                 \
        line_kernel<l, t><<<g, kThreads, lds, s>>>(spec1, spec0, so, sn, hty, twM, N, prm, sz, br); \
        return 0;                                                                                        \
    }
    ADMM_LT_CASES(X)
#undef X
    return -1;
}

// planes: per branch; ngb: plane groups per branch (grid y = branches x ngb), 0: one branch
int launch_iso_a(int L, int T, dim3 g, size_t lds, hipStream_t s, const float2* spec1, const float* so, float* sn,
                 const float* fmap, float* part, const float2* twM, int N, int planes, int G, int sz, int ngb = 0) {
#define X(l, t)                                                                                             \
    if (L == l && T == t) {                                                                                 \
        set_lds(iso_a_kernel<l, t>, lds);                                                                   \
        iso_a_kernel<l, t><<<g, kThreads, lds, s>>>(spec1, so, sn, fmap, part, twM, N, planes, G, sz, ngb); \
        return 0;                                                                                           \
    }
    ADMM_LT_CASES(X)
#undef X
    return -1;
}

int launch_iso_b(int L, int T, dim3 g, size_t lds, hipStream_t s, const float* sn, const float* fmap,
                 const float* hty, float2* spec0, const float2* twM, int N, const float* prm,
                 const Branches& br = kOneSolve) {
#define X(l, t)                                                                               \
    if (L == l && T == t) {                                                                   \
        set_lds(iso_b_kernel<l, t>, lds);                                                     \
        iso_b_kernel<l, t><<<g, kThreads, lds, s>>>(sn, fmap, hty, spec0, twM, N, prm, br);  \
        return 0;                                                                             \
    }
    ADMM_LT_CASES(X)
#undef X
    return -1;
}

template <int MUL, bool SAVE, bool ACCQ, int YH = YH_NONE>
int launch_column_t(int N, dim3 g, size_t lds, hipStream_t s, const float2* src, float2* dst, const float* C,
                    const float2* G, const float2* twN, int L, int KB, float cs, float2* vsave, double* Qp,
                    const Branches& br, float2* yh = nullptr) {
    const int nt = column_threads(N);
#define X(v)                                                                                                   \
    if (N == v && nt == kThreads) {                                                                            \
        set_lds(column_kernel<v, MUL, SAVE, ACCQ, kThreads, YH>, lds);                                         \
        column_kernel<v, MUL, SAVE, ACCQ, kThreads, YH><<<g, kThreads, lds, s>>>(src, dst, C, G, twN, L, KB, cs,  \
                                                                                  vsave, Qp, br, yh);             \
        return 0;                                                                                              \
    }
    ADMM_N_CASES(X)
#undef X
#define X(v)                                                                                                   \
    if (N == v && nt == 512) {                                                                                 \
        set_lds(column_kernel<v, MUL, SAVE, ACCQ, 512, YH>, lds);                                              \
        column_kernel<v, MUL, SAVE, ACCQ, 512, YH><<<g, 512, lds, s>>>(src, dst, C, G, twN, L, KB, cs, vsave, Qp, br, \
                                                                       yh);                                        \
        return 0;                                                                                              \
    }
    X(256) X(512) X(1024)
#undef X
#define X(v)                                                                                                   \
    if (N == v && nt == 1024) {                                                                                \
        set_lds(column_kernel<v, MUL, SAVE, ACCQ, 1024, YH>, lds);                                             \
        column_kernel<v, MUL, SAVE, ACCQ, 1024, YH><<<g, 1024, lds, s>>>(src, dst, C, G, twN, L, KB, cs, vsave, Qp,  \
                                                                         br, yh);                                   \
        return 0;                                                                                              \
    }
    X(256) X(512) X(1024)
#undef X
    return -1;
}

// mode: 0 = x-update C, 1 = conj(Sigma_c) (H^T), 2 = Sigma_c (H), 3 = C + save spectrum, 4 = C + accumulate Q;
// 5 = Y_h = cs conj(Sigma_c) F y stored to yh (G NULL: Y_h = cs F y), no inverse; 6 = + yh, x C; 7 = + yh, save, x C
// (admm_kernels.hip YH_STORE / YH_ADD: H^T y in the spectral domain); br: several branches (C per branch, br.tab_f
// floats apart)
int launch_column(int N, int mode, dim3 g, size_t lds, hipStream_t s, const float2* src, float2* dst,
                  const float* C, const float2* G, const float2* twN, int L, int KB, float cs,
                  float2* vsave = nullptr, double* Qp = nullptr, const Branches& br = kOneSolve, float2* yh = nullptr) {
    switch (mode) {
        case 5: return launch_column_t<1, false, false, YH_STORE>(N, g, lds, s, src, dst, C, G, twN, L, KB, cs, vsave, Qp, br, yh);
        case 6: return launch_column_t<0, false, false, YH_ADD>(N, g, lds, s, src, dst, C, G, twN, L, KB, cs, vsave, Qp, br, yh);
        case 7: return launch_column_t<0, true, false, YH_ADD>(N, g, lds, s, src, dst, C, G, twN, L, KB, cs, vsave, Qp, br, yh);
        case 0: return launch_column_t<0, false, false>(N, g, lds, s, src, dst, C, G, twN, L, KB, cs, vsave, Qp, br);
        case 1: return launch_column_t<1, false, false>(N, g, lds, s, src, dst, C, G, twN, L, KB, cs, vsave, Qp, br);
        case 2: return launch_column_t<2, false, false>(N, g, lds, s, src, dst, C, G, twN, L, KB, cs, vsave, Qp, br);
        case 3: return launch_column_t<0, true, false>(N, g, lds, s, src, dst, C, G, twN, L, KB, cs, vsave, Qp, br);
        case 4: return launch_column_t<0, false, true>(N, g, lds, s, src, dst, C, G, twN, L, KB, cs, vsave, Qp, br);
    }
    return -1;
}

// ---- generic-size path (admm_generic.hip) ----------------------------------------------------
admm::gen::FPlan make_fplan(int n) {
    admm::gen::FPlan p{};
    p.n = n;
    int m = n;
    auto add = [&](int r) { p.r[p.nf++] = r; m /= r; };
    while (m % 8 == 0) add(8);
    if (m % 4 == 0) add(4);
    if (m % 2 == 0) add(2);
    while (m % 3 == 0) add(3);
    while (m % 5 == 0) add(5);
    for (int f = 7; f * f <= m; f += 2)
        while (m % f == 0) add(f);
    if (m > 1) add(m);
    return p;
}

int run_forward_generic(Launcher& ln, const float* y, float* x_out, int M, int N, size_t planes, int kh,
                        int iso, int maxit, unsigned char* ws, const Layout& lay,
                        const Traj& tr, const admm_batch_reducer* red, int path);

// the caller's cross-shard sum of an M x N map (isotropic prox over a sharded batch)
int call_reducer(const admm_batch_reducer* red, float* buf, size_t count, hipStream_t s) {
    const int r = red->fn(buf, count, reinterpret_cast<void*>(s), red->user);
    if (r != 0) return fail(ADMM_E_REDUCER, "batch reducer returned %d", r);
    return ADMM_OK;
}

// Isotropic CU-resident solve (ADMM_PATH_RESIDENT_ISO): iteration k is one resident_iso_kernel launch (s_k, f_k ->
// s_{k+1}, q per plane; x at the last), then the 2-pass path's norm over the planes' q (iso_r, or for a sharded
// batch the shard sum, the caller's all-reduce and the factor) -> f_{k+1} (and |s_{k+1}| when recording).
// Recording: s_{k+1} into trajectory slot k, read back from slot k - 1 -- the natural layout the 2-pass and
// runtime-length isotropic sweeps read.  q: planes x M x N floats (a spectrum buffer, free after PREP).
int run_resident_iso(Launcher& ln, int M, int N, size_t planes, const float* hty, float* sbuf0, float* q, float* fmap,
                     float* x_out, const float* Ct, const float2* twM, const float2* twN, const float* prm, int maxit,
                     const Traj& tr, const admm_batch_reducer* red) {
    hipStream_t s = ln.s;
    const size_t MN = (size_t)M * N, sstride = planes * 2 * MN;
    const int nb = (int)((MN + 63) / 64);   // 64 pixels per block (group_sum)
    const dim3 gr(nb < 2048 ? nb : 2048);
    for (int k = 0; k < maxit; ++k) {
        const float* sin = tr.s && k >= 1 ? tr.s + (size_t)(k - 1) * sstride : sbuf0;
        float* sout = tr.s ? tr.s + (size_t)k * sstride : sbuf0;
        int rc = ln.run(ADMM_K_PLANE, [&] {
            return admm::rs::launch_iso(M, N, planes, s, hty, sin, sout, fmap, q, x_out, Ct, twM, twN, prm, k, maxit);
        });
        if (rc) return rc;
        if (k + 1 == maxit) break;
        float* nrm_out = tr.nrm ? tr.nrm + (size_t)k * MN : nullptr;
        if (red) {
            rc = ln.run(ADMM_K_NORM, [&] {
                hipLaunchKernelGGL(admm::iso_sum_kernel, gr, dim3(kThreads), 0, s, q, fmap, (int)planes, MN);
            });
            if (rc) return rc;
            rc = call_reducer(red, fmap, MN, s);
            if (rc) return rc;
            rc = ln.run(ADMM_K_NORM, [&] {
                hipLaunchKernelGGL(admm::iso_fin_kernel, gr, dim3(kThreads), 0, s, fmap, MN, prm, nrm_out);
            });
        } else {
            rc = ln.run(ADMM_K_NORM, [&] {
                hipLaunchKernelGGL(admm::iso_r_kernel, gr, dim3(kThreads), 0, s, q, fmap, (int)planes, MN, prm, nrm_out);
            });
        }
        if (rc) return rc;
    }
    return ADMM_OK;
}

int run_forward(Launcher& ln, const float* y, float* x_out, int M, int N, size_t planes, const float* h, int kh,
                int kw, const admm::ScalarSrc& sc, int iso, int maxit, unsigned char* ws, const Layout& lay,
                const Traj& tr, const admm_batch_reducer* red, int fwd_path, bool tables) {
    hipStream_t s = ln.s;
    int rc = ADMM_OK;
    const size_t MN = (size_t)M * N;
    float2* twM = reinterpret_cast<float2*>(ws + lay.twM);
    float2* twN = reinterpret_cast<float2*>(ws + lay.twN);
    float* Ct = reinterpret_cast<float*>(ws + lay.C);
    float2* Gt = kh > 0 ? reinterpret_cast<float2*>(ws + lay.G) : nullptr;
    float* hty = kh > 0 ? reinterpret_cast<float*>(ws + lay.hty) : const_cast<float*>(y);
    float* sbuf[2] = {reinterpret_cast<float*>(ws + lay.sA), reinterpret_cast<float*>(ws + lay.sB)};
    float2* spec0 = reinterpret_cast<float2*>(ws + lay.spec0);
    float2* spec1 = reinterpret_cast<float2*>(ws + lay.spec1);
    const int L = M / 2;
    float* prm = reinterpret_cast<float*>(ws + lay.prm);   // tau = lambda / rho (ops.jl:20), rho, lambda
    double2* SigT = tr.sig;

    if (tables) rc = ln.run(ADMM_K_SETUP, [&] {
        const size_t lds = (size_t)(M + N) * 16 + (kh * kw <= admm::kSetupPsfLds ? (size_t)kh * kw * 4 : 0);
        const int nb = (int)(((size_t)(L + 1) * N * (kh > 0 ? admm::kSetupSplit : 1) + kThreads - 1) / kThreads);
        const int grid = nb < 1024 ? (nb < 1 ? 1 : nb) : 1024;
        set_lds(admm::setup_kernel, lds);
        hipLaunchKernelGGL(admm::setup_kernel, dim3(grid), dim3(kThreads), lds, s, twM, twN, Ct, Gt, h, kh, kw, M,
                           N, sc, prm, SigT);
    });
    if (rc) return rc;
    if (maxit == 0) {
        hipError_t e = hipMemsetAsync(x_out, 0, planes * MN * 4, s);
        if (e != hipSuccess) return fail(ADMM_E_HIP, "hipMemsetAsync: %s", hipGetErrorString(e));
        return ADMM_OK;
    }

    const int path = fwd_path;
    if (generic_shape(M, N)) {   // ADMM_PATH_RESIDENT (smooth sides), _SMOOTH, _RUNTIME: the runtime-length layout
        return run_forward_generic(ln, y, x_out, M, N, planes, kh, iso, maxit, ws, lay, tr, red, path);
    }
    if (path == ADMM_PATH_FUSED) {
        // one workgroup per plane runs all K iterations (plane_kernel.hip); lane-native H^T y in
        // spec0, lane-native s in sA -- or, recording a trajectory, s_k in its own slot of tr.s
        namespace pk = admm::plane;
        void* ptab = ws + lay.F;
        if (tables) rc = ln.run(ADMM_K_SETUP, [&] { return pk::launch_tables(Ct, Gt, ptab, s); });
        if (rc) return rc;
        rc = ln.run(ADMM_K_PLANE, [&] {
            return pk::launch_plane(y, x_out, ptab, kh > 0, spec0, reinterpret_cast<float4*>(sbuf[0]), prm, maxit,
                                   planes, s, tr.m ? nullptr : reinterpret_cast<float4*>(tr.s), nullptr, tr.m);
        });
        return rc;
    }
    if (path == ADMM_PATH_FUSED_ISO) {
        // isotropic at 256 x 256: the split-iteration per-plane kernels (plane_iso.hip), the spectrum
        // resident in the CU; per iteration one plane256_iso_kernel and one iso_norm_kernel (batch norm)
        namespace pk = admm::plane;
        void* ptab = ws + lay.F;
        if (tables) rc = ln.run(ADMM_K_SETUP, [&] { return pk::launch_tables(Ct, Gt, ptab, s); });
        if (rc) return rc;
        float2* fl = reinterpret_cast<float2*>(ws + lay.fmap);
        float2* ql = reinterpret_cast<float2*>(spec1);
        // recording: s_{k+1} into trajectory slot k, |s_{k+1}| into norm slot k (lane-native)
        float4* st = reinterpret_cast<float4*>(tr.iso_lane ? tr.s : sbuf[0]);
        const size_t tslot = tr.iso_lane ? planes * MN / 2 : 0;   // float4 per slot
        for (int k = 0; k < maxit; ++k) {
            rc = ln.run(ADMM_K_PLANE, [&] {
                return pk::launch_plane_iso(y, x_out, ptab, kh > 0, spec0, st + (k > 0 ? (size_t)(k - 1) * tslot : 0),
                                            st + (size_t)k * tslot, fl, ql, prm, k, maxit, planes, s);
            });
            if (rc) return rc;
            if (k + 1 < maxit) {
                float2* nr = tr.iso_lane ? reinterpret_cast<float2*>(tr.nrm + (size_t)k * MN) : nullptr;
                if (red) {
                    // sharded batch: this shard's sums, the caller's all-reduce of the M x N map, then f
                    float2* sm = reinterpret_cast<float2*>(ws + lay.part);
                    rc = ln.run(ADMM_K_NORM, [&] { return pk::launch_iso_norm(ql, fl, nr, prm, planes, s, nullptr, sm); });
                    if (rc) return rc;
                    rc = call_reducer(red, reinterpret_cast<float*>(sm), MN, s);
                    if (rc) return rc;
                    rc = ln.run(ADMM_K_NORM, [&] {
                        return pk::launch_iso_norm(ql, fl, nr, prm, planes, s, nullptr, nullptr, sm);
                    });
                } else {
                    rc = ln.run(ADMM_K_NORM, [&] { return pk::launch_iso_norm(ql, fl, nr, prm, planes, s); });
                }
                if (rc) return rc;
            }
        }
        return ADMM_OK;
    }
    const int T = line_T(M, N);
    const int KB = column_KB(M, N);
    // the per-iteration line update runs 4-line blocks at 512-point lines (its just-in-time loads let 4 of
    // them share a CU, admm_kernels.hip line_kernel); the one-off line transforms keep T
    // 512-point lines: 8-line update blocks of 512 threads (round 5, tools/c4_line_sweep.sh: line pass 1.217 ->
    // 1.196 ms at c4; 4 lines x 256 threads was round 1's choice; 16 x 1024, 4 x 512 and 8 x 1024 slower:
    // profiles/r05_c4_line_sweep.jsonl)
    const int Tu = (M == 512 && T > 4) ? 8 : T;
    const int nTu = (M == 512 && Tu == 8) ? 512 : kThreads;
    const size_t llds = line_lds(M, Tu), flds = fwdinv_lds(M, T), clds = column_lds(N, KB);
    float* fmap = iso ? reinterpret_cast<float*>(ws + lay.fmap) : nullptr;
    float* part = iso ? reinterpret_cast<float*>(ws + lay.part) : nullptr;
    const size_t np = planes;
    const dim3 gl(N / T, (unsigned)np), gc(L / KB, (unsigned)np);
    if (path == ADMM_PATH_RESIDENT || path == ADMM_PATH_RESIDENT_ISO) {
        // power-of-two sides admm_resident.hip compiled: one workgroup per plane runs all K iterations (s_k into
        // the trajectory slots when recording, natural layout, as the 2-pass sweep reads them); H^T y from the
        // 2-pass PREP kernels (line, column x conj(Sigma_c), line), the first line spectrum formed in the kernel
        if (kh > 0) {
            rc = ln.run(ADMM_K_PREP, [&] { return launch_line_fwd(L, T, gl, flds, s, y, spec0, twM, N); });
            if (rc) return rc;
            rc = ln.run(ADMM_K_PREP, [&] { return launch_column(N, 1, gc, clds, s, spec0, spec1, Ct, Gt, twN, L, KB, 1.0f); });
            if (rc) return rc;
            rc = ln.run(ADMM_K_PREP, [&] { return launch_line_inv(L, T, gl, flds, s, spec1, hty, twM, N); });
            if (rc) return rc;
        }
        if (path == ADMM_PATH_RESIDENT_ISO)
            return run_resident_iso(ln, M, N, planes, hty, sbuf[0], reinterpret_cast<float*>(spec1), fmap, x_out, Ct, twM,
                                    twN, prm, maxit, tr, red);
        return ln.run(ADMM_K_PLANE, [&] {
            return admm::rs::launch(M, N, planes, s, hty, sbuf[0], sbuf[1], tr.s, np * 2 * MN, x_out, Ct, twM, twN, prm,
                                    maxit);
        });
    }
    // PREP: Y_h = F(H^T y) = conj(Sigma_c) F y as a 2-D packed spectrum straight from F y (line transform, column
    // transform x conj(Sigma_c)), never H^T y in space: every iteration adds it to the spectrum of rho D^T w in
    // the column pass, so the per-iteration fp32 transforms carry only rho D^T w (x 16x, y_bar / h_bar ~2-9x closer
    // to the fp64 oracle than with H^T y added before the line transform; DESIGN.md s1 "H^T y in the spectrum").
    // Iteration 1 (w = 0) transforms a zero line spectrum and adds Y_h.
    float2* yh = reinterpret_cast<float2*>(ws + lay.hty);   // the workspace's H^T y slot holds Y_h on this path
    rc = ln.run(ADMM_K_PREP, [&] { return launch_line_fwd(L, T, gl, flds, s, y, spec0, twM, N); });
    if (rc) return rc;
    rc = ln.run(ADMM_K_PREP, [&] {
        return launch_column(N, 5, gc, clds, s, spec0, spec1, Ct, kh > 0 ? Gt : nullptr, twN, L, KB,
                             kh > 0 ? (float)MN : 1.0f, nullptr, nullptr, kOneSolve, yh);
    });
    if (rc) return rc;
    {
        hipError_t e = hipMemsetAsync(spec0, 0, np * MN * 4, s);
        if (e != hipSuccess) return fail(ADMM_E_HIP, "hipMemsetAsync: %s", hipGetErrorString(e));
    }
    const size_t sstride = np * 2 * MN;   // one trajectory slot of s
    for (int it = 1; it <= maxit; ++it) {
        float2* vsave = tr.v ? tr.v + (size_t)(it - 1) * np * N * L : nullptr;
        rc = ln.run(ADMM_K_COLUMN, [&] {
            return launch_column(N, vsave ? 7 : 6, gc, clds, s, spec0, spec1, Ct, Gt, twN, L, KB, 1.0f, vsave, nullptr,
                                 kOneSolve, yh);
        });
        if (rc) return rc;
        if (it < maxit && !iso) {
            float* so;
            float* sn;
            if (tr.s) {
                so = it >= 2 ? tr.s + (size_t)(it - 2) * sstride : sbuf[0];
                sn = tr.s + (size_t)(it - 1) * sstride;
            } else {
                so = (it & 1) ? sbuf[1] : sbuf[0];   // iteration 1 reads nothing (s_zero)
                sn = (it & 1) ? sbuf[0] : sbuf[1];
            }
            rc = ln.run(ADMM_K_LINE, [&] {
                return launch_line(L, Tu, dim3(N / Tu, (unsigned)np), llds, s, spec1, spec0, so, sn, nullptr, twM, N, prm,
                            it == 1 ? 1 : 0, nTu);
            });
        } else if (it < maxit) {
            // isotropic: s is written in place (no halo reads of s in ISO_A); with a trajectory each
            // iteration writes its own slot and the batch norm is kept too
            float* so = sbuf[0];
            float* sn = sbuf[0];
            if (tr.s) {
                so = it >= 2 ? tr.s + (size_t)(it - 2) * sstride : sbuf[0];
                sn = tr.s + (size_t)(it - 1) * sstride;
            }
            float* nrm_out = tr.nrm ? tr.nrm + (size_t)(it - 1) * MN : nullptr;
            const int ng = iso_ngroups(np);
            rc = ln.run(ADMM_K_LINE, [&] {
                return launch_iso_a(L, T, dim3(N / T, ng), iso_a_lds(M, T), s, spec1, so, sn, fmap, part, twM, N, (int)np,
                             iso_group(np), it == 1 ? 1 : 0);
            });
            if (rc) return rc;
            const int nb = (int)((MN + 63) / 64);   // 64 pixels per block (group_sum)
            const dim3 gr(nb < 2048 ? nb : 2048);
            if (red) {
                // sharded batch: per-shard sum -> caller's all-reduce -> BT factor
                rc = ln.run(ADMM_K_NORM, [&] {
                    hipLaunchKernelGGL(admm::iso_sum_kernel, gr, dim3(kThreads), 0, s, part, fmap, ng, MN);
                });
                if (rc) return rc;
                rc = call_reducer(red, fmap, MN, s);
                if (rc) return rc;
                rc = ln.run(ADMM_K_NORM, [&] {
                    hipLaunchKernelGGL(admm::iso_fin_kernel, gr, dim3(kThreads), 0, s, fmap, MN, prm, nrm_out);
                });
            } else {
                rc = ln.run(ADMM_K_NORM, [&] {
                    hipLaunchKernelGGL(admm::iso_r_kernel, gr, dim3(kThreads), 0, s, part, fmap, ng, MN, prm, nrm_out);
                });
            }
            if (rc) return rc;
            rc = ln.run(ADMM_K_LINE, [&] {
                return launch_iso_b(L, T, gl, iso_b_lds(M, T), s, sn, fmap, nullptr, spec0, twM, N, prm);
            });
        } else {
            rc = ln.run(ADMM_K_FINAL, [&] { return launch_line_inv(L, T, gl, flds, s, spec1, x_out, twM, N); });
        }
        if (rc) return rc;
    }
    return ADMM_OK;
}

int run_forward_generic(Launcher& ln, const float* y, float* x_out, int M, int N, size_t planes, int kh,
                        int iso, int maxit, unsigned char* ws, const Layout& lay,
                        const Traj& tr, const admm_batch_reducer* red, int path) {
    namespace g = admm::gen;
    hipStream_t s = ln.s;
    int rc = ADMM_OK;
    const size_t MN = (size_t)M * N;
    const int H = M / 2 + 1;
    const float2* twM = reinterpret_cast<float2*>(ws + lay.twM);
    const float2* twN = reinterpret_cast<float2*>(ws + lay.twN);
    const float* Ct = reinterpret_cast<float*>(ws + lay.C);
    const float2* Gt = kh > 0 ? reinterpret_cast<float2*>(ws + lay.G) : nullptr;
    const float* hty = kh > 0 ? reinterpret_cast<float*>(ws + lay.hty) : y;
    float* sbuf[2] = {reinterpret_cast<float*>(ws + lay.sA), reinterpret_cast<float*>(ws + lay.sB)};
    float2* spec0 = reinterpret_cast<float2*>(ws + lay.spec0);
    float2* spec1 = reinterpret_cast<float2*>(ws + lay.spec1);
    float* xg = reinterpret_cast<float*>(ws + lay.xg);
    float* fmap = iso ? reinterpret_cast<float*>(ws + lay.fmap) : nullptr;
    float* part = iso ? reinterpret_cast<float*>(ws + lay.part) : nullptr;
    const float* prm = reinterpret_cast<const float*>(ws + lay.prm);
    const g::FPlan pM = make_fplan(M), pN = make_fplan(N);
    const int T = gen_T(M, N), KB = gen_KB(M, N);
    const dim3 gl(gen_nb(N, T), (unsigned)planes), gc((H + KB - 1) / KB, (unsigned)planes);
    const size_t lfw = gen_lds_line(M, T, false);                    // line_fwd / line_inv
    const size_t lup = gen_lds_line(M, T, true);                     // line_upd / iso_b
    const size_t lcol = gen_lds_col(N, KB);
    set_lds(g::line_fwd_kernel, lfw);
    set_lds(g::line_inv_kernel, lfw);
    set_lds(g::line_upd_kernel, lup);
    set_lds(g::iso_b_kernel, lup);
    set_lds(g::column_kernel, lcol);
    // compile-time-plan kernels where this build has the length (admm_smooth.hip): the column pass needs
    // N, the line passes M
    const bool smc = opt(ADMM_OPT_SMOOTH) != 0 && admm::sm::has_length(N);
    const bool sml = opt(ADMM_OPT_SMOOTH) != 0 && admm::sm::has_length(M);
    auto line_fwd = [&](const float* src, float2* dst) {
        return ln.run(ADMM_K_PREP, [&] {
            if (sml) return admm::sm::launch_line_fwd(M, N, planes, s, src, dst, twM);
            hipLaunchKernelGGL(g::line_fwd_kernel, gl, dim3(256), lfw, s, src, dst, twM, pM, N, T);
            return 0;
        });
    };
    // CU-resident solve (admm_resident.hip): anisotropic, no dim-2 spectra or isotropic norms recorded; it
    // forms the first line spectrum itself, so PREP only produces H^T y
    const bool res = path == ADMM_PATH_RESIDENT || path == ADMM_PATH_RESIDENT_ISO;   // plan_paths
    // the 2-pass kernels take H^T y in the spectral domain: Y_h = conj(Sigma_c) F y (with a PSF) stored once as the
    // column pass's 2-D spectrum and added to every iteration's spectrum of rho D^T w
    float2* yh = reinterpret_cast<float2*>(ws + lay.hty);
    if (!res) {
        rc = line_fwd(y, spec0);
        if (rc) return rc;
        rc = ln.run(ADMM_K_PREP, [&] {
            hipLaunchKernelGGL(g::column_kernel, gc, dim3(256), lcol, s, spec0, spec1, Ct, Gt, twN, pN, H, KB, 32 | 1,
                               kh > 0 ? (float)MN : 1.0f, (float2*)nullptr, (double*)nullptr, yh);
            return 0;
        });
        if (rc) return rc;
        hipError_t e = hipMemsetAsync(spec0, 0, planes * (size_t)H * N * 8, s);   // iteration 1: w = 0
        if (e != hipSuccess) return fail(ADMM_E_HIP, "hipMemsetAsync: %s", hipGetErrorString(e));
    }
    // PREP of the resident solves: H^T y in space (with a PSF: F^-1 conj(Sigma_c) F y, ops.jl:71-81)
    if (res && kh > 0) {
        rc = line_fwd(y, spec0);
        if (rc) return rc;
    }
    if (res && kh > 0) {
        rc = ln.run(ADMM_K_PREP, [&] {
            if (smc) return admm::sm::launch_column(M, N, planes, s, spec0, spec1, Ct, Gt, twN, 1.0f, 1, opt(ADMM_OPT_SMOOTH));
            hipLaunchKernelGGL(g::column_kernel, gc, dim3(256), lcol, s, spec0, spec1, Ct, Gt, twN, pN, H, KB, 1, 1.0f);
            return 0;
        });
        if (rc) return rc;
        rc = ln.run(ADMM_K_PREP, [&] {
            if (sml) return admm::sm::launch_line_inv(M, N, planes, s, spec1, const_cast<float*>(hty), twM);
            hipLaunchKernelGGL(g::line_inv_kernel, gl, dim3(256), lfw, s, spec1, const_cast<float*>(hty), twM, pM, N, T);
            return 0;
        });
        if (rc) return rc;
    }
    const int ng = iso_ngroups(planes);
    const size_t sstride = planes * 2 * MN;   // one trajectory slot of s
    if (path == ADMM_PATH_RESIDENT_ISO)
        return run_resident_iso(ln, M, N, planes, hty, sbuf[0], reinterpret_cast<float*>(spec1), fmap, x_out, Ct, twM, twN,
                                prm, maxit, tr, red);
    if (res) {
        return ln.run(ADMM_K_PLANE, [&] {
            return admm::rs::launch(M, N, planes, s, hty, sbuf[0], sbuf[1], tr.s, sstride, x_out, Ct, twM, twN, prm, maxit);
        });
    }
    for (int it = 1; it <= maxit; ++it) {
        // trajectory for h_bar: the dim-2 spectrum of iteration it before the multiply
        float2* vsave = tr.v ? tr.v + (size_t)(it - 1) * planes * N * H : nullptr;
        rc = ln.run(ADMM_K_COLUMN, [&] {
            if (smc && !vsave)
                return admm::sm::launch_column(M, N, planes, s, spec0, spec1, Ct, Gt, twN, 1.0f, 0, opt(ADMM_OPT_SMOOTH), yh);
            hipLaunchKernelGGL(g::column_kernel, gc, dim3(256), lcol, s, spec0, spec1, Ct, Gt, twN, pN, H, KB,
                               (vsave ? 4 : 0) | 16, 1.0f, vsave, (double*)nullptr, yh);
            return 0;
        });
        if (rc) return rc;
        const bool last = it == maxit;
        rc = ln.run(last ? ADMM_K_FINAL : ADMM_K_LINE, [&] {
            if (sml) return admm::sm::launch_line_inv(M, N, planes, s, spec1, last ? x_out : xg, twM);
            hipLaunchKernelGGL(g::line_inv_kernel, gl, dim3(256), lfw, s, spec1, last ? x_out : xg, twM, pM, N, T);
            return 0;
        });
        if (rc) return rc;
        if (last) break;
        if (!iso) {
            float* so = (it & 1) ? sbuf[1] : sbuf[0];   // iteration 1 reads nothing (first)
            float* sn = (it & 1) ? sbuf[0] : sbuf[1];
            if (tr.s) {   // s_it into its own trajectory slot
                so = it >= 2 ? tr.s + (size_t)(it - 2) * sstride : sbuf[0];
                sn = tr.s + (size_t)(it - 1) * sstride;
            }
            rc = ln.run(ADMM_K_LINE, [&] {
                if (sml) return admm::sm::launch_line_upd(M, N, planes, s, xg, so, sn, nullptr, spec0, twM, prm, it == 1 ? 1 : 0);
                hipLaunchKernelGGL(g::line_upd_kernel, gl, dim3(256), lup, s, xg, so, sn, (const float*)nullptr, spec0, twM,
                                   pM, N, T, prm, it == 1 ? 1 : 0);
                return 0;
            });
            if (rc) return rc;
            continue;
        }
        float* sa = sbuf[0];
        const float* s_in = sbuf[0];
        if (tr.s) {
            s_in = it >= 2 ? tr.s + (size_t)(it - 2) * sstride : sbuf[0];
            sa = tr.s + (size_t)(it - 1) * sstride;
        }
        float* nrm_out = tr.nrm ? tr.nrm + (size_t)(it - 1) * MN : nullptr;
        rc = ln.run(ADMM_K_LINE, [&] {
            hipLaunchKernelGGL(g::iso_a_kernel, dim3(gen_nb(N, T), ng), dim3(256), (size_t)T * M * 4, s, xg, s_in, sa, fmap,
                               part, M, N, (int)planes, iso_group(planes), T, it == 1 ? 1 : 0);
        });
        if (rc) return rc;
        const int nb = (int)((MN + 63) / 64);   // 64 pixels per block (group_sum)
        const dim3 gr(nb < 2048 ? nb : 2048);
        if (red) {
            rc = ln.run(ADMM_K_NORM, [&] {
                hipLaunchKernelGGL(admm::iso_sum_kernel, gr, dim3(kThreads), 0, s, part, fmap, ng, MN);
            });
            if (rc) return rc;
            rc = call_reducer(red, fmap, MN, s);
            if (rc) return rc;
            rc = ln.run(ADMM_K_NORM, [&] {
                hipLaunchKernelGGL(admm::iso_fin_kernel, gr, dim3(kThreads), 0, s, fmap, MN, prm, nrm_out);
            });
        } else {
            rc = ln.run(ADMM_K_NORM, [&] {
                hipLaunchKernelGGL(admm::iso_r_kernel, gr, dim3(kThreads), 0, s, part, fmap, ng, MN, prm, nrm_out);
            });
        }
        if (rc) return rc;
        rc = ln.run(ADMM_K_LINE, [&] {
            hipLaunchKernelGGL(g::iso_b_kernel, gl, dim3(256), lup, s, sa, fmap, (const float*)nullptr, spec0, twM, pM, N, T,
                               prm);
        });
        if (rc) return rc;
    }
    return ADMM_OK;
}

// out[c] = sum over the n rows of column c of part (n x w row-major), in a fixed order
void launch_reduce_cols(hipStream_t s, const double* part, double* out, int n, int w, double* tmp) {
    const int chunk = 2048;
    const int parts = (n + chunk - 1) / chunk;
    if (parts <= 1) {
        hipLaunchKernelGGL(admm::reduce_cols_kernel, dim3(w), dim3(kThreads), 0, s, part, out, n, w);
        return;
    }
    const int ch = (n + (parts < kRedParts ? parts : kRedParts) - 1) / (parts < kRedParts ? parts : kRedParts);
    const int g = (n + ch - 1) / ch;
    hipLaunchKernelGGL(admm::reduce_cols_part_kernel, dim3(w, g), dim3(kThreads), 0, s, part, tmp, n, w, ch);
    hipLaunchKernelGGL(admm::reduce_cols_kernel, dim3(w), dim3(kThreads), 0, s, tmp, out, g, w);
}

int launch_line_adj(int L, int T, dim3 g, size_t lds, hipStream_t s, const float2* spec1, const float* sk1,
                    const float* sk, const float* xK, const float* sb_in, float* sb_out, float* vsum, float2* spec0,
                    double* part, const float2* twM, int N, const float* prm, int first_k, int last_k, bool ln,
                    const Branches& br = kOneSolve, size_t pbs = 0) {
    if (ln) {   // trajectory in the fused kernel's lane-native layout (M = 256)
#define X(l, t)                                                                                                \
        if (L == l && T == t) {                                                                                \
            set_lds(line_adj_kernel<l, t, true>, lds);                                                         \
            line_adj_kernel<l, t, true><<<g, kThreads, lds, s>>>(spec1, sk1, sk, xK, sb_in, sb_out, vsum, spec0, \
                                                                  part, twM, N, prm, first_k, last_k);    \
            return 0;                                                                                          \
        }
        X(128, 2) X(128, 4) X(128, 8) X(128, 16)
#undef X
        return -1;
    }
#define X(l, t)                                                                                                \
    if (L == l && T == t) {                                                                                    \
        set_lds(line_adj_kernel<l, t>, lds);                                                                   \
        line_adj_kernel<l, t><<<g, kThreads, lds, s>>>(spec1, sk1, sk, xK, sb_in, sb_out, vsum, spec0, part, twM, \
                                                        N, prm, first_k, last_k, br, pbs);               \
        return 0;                                                                                              \
    }
    ADMM_LT_CASES(X)
#undef X
    return -1;
}

// br / ngb / pbs: several branches (planes per branch, plane groups per branch, doubles between the branches'
// partial-row blocks)
int launch_iso_adj_a(int L, int T, dim3 g, size_t lds, hipStream_t s, const float2* spec1, const float* sk1,
                     const float* sk, const float* xK, const float* nrm1, const float* sb_in, float* wbar, float* vsum,
                     float* rpartial, double* part, const float2* twM, int N, int planes, int G, const float* prm,
                     int first_k, int last_k, const Branches& br = kOneSolve, int ngb = 0, size_t pbs = 0) {
#define X(l, t)                                                                                                 \
    if (L == l && T == t) {                                                                                     \
        set_lds(iso_adj_a_kernel<l, t>, lds);                                                                   \
        iso_adj_a_kernel<l, t><<<g, kThreads, lds, s>>>(spec1, sk1, sk, xK, nrm1, nullptr, sb_in, wbar, vsum,  \
                                                         rpartial, part, twM, N, planes, G, prm, first_k,  \
                                                         last_k, br, ngb, pbs);                                 \
        return 0;                                                                                               \
    }
    ADMM_LT_CASES(X)
#undef X
    return -1;
}

int launch_iso_adj_b(int L, int T, dim3 g, size_t lds, hipStream_t s, const float* wbar, const float* sb_in,
                     const float* sk1, const float* nrm1, const float* Rmap, float* sb_out, float2* spec0,
                     const float2* twM, int N, const float* prm, const Branches& br = kOneSolve) {
#define X(l, t)                                                                                                 \
    if (L == l && T == t) {                                                                                     \
        set_lds(iso_adj_b_kernel<l, t>, lds);                                                                   \
        iso_adj_b_kernel<l, t><<<g, kThreads, lds, s>>>(wbar, sb_in, sk1, nrm1, Rmap, sb_out, spec0, twM, N,    \
                                                         prm, br);                                              \
        return 0;                                                                                               \
    }
    ADMM_LT_CASES(X)
#undef X
    return -1;
}

int launch_backward(int phases, const float* y, const float* x_bar, float* y_bar, float* h_bar, float* lambda_bar,
                    float* rho_bar, int M, int N, size_t planes, const float* h, int kh, int kw,
                    const admm::ScalarSrc& sc, int iso, int maxit, float* x_out, void* workspace, void* stream,
                    const admm_batch_reducer* red, const PathPlan& plan, const BwdLayout& bl) {
    int rc = ADMM_OK;
    const bool want_h = plan.want_h;
    const bool ln_traj = plan.ln_traj;
    const bool use_masks = plan.masks;
    const bool iso_lane = plan.iso_lane;   // the fused isotropic sweep (no mask bits: s itself is needed)
    unsigned char* ws = static_cast<unsigned char*>(workspace);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    Launcher ln{s, g_prof.on, {}};
    const size_t MN = (size_t)M * N;
    const int L = M / 2;
    const bool gen = generic_shape(M, N);   // runtime-length path (admm_generic.hip, admm_generic_bwd.hip)
    const int T = gen ? gen_T(M, N) : bwd_line_T(M, N, iso != 0);
    const int KB = gen ? gen_KB(M, N) : column_KB(M, N);
    float* prm = reinterpret_cast<float*>(ws + bl.f.prm);
    const int K = maxit;
    if (!x_out || (reinterpret_cast<uintptr_t>(x_out) & 15))
        return fail(ADMM_E_INVALID, "x_out (forward output of the recomputed solve) must be a 16-byte aligned device pointer");
    float* xK = x_out;
    hipError_t e;
#define HIPCHK(call)                                                                           \
    do {                                                                                       \
        e = (call);                                                                            \
        if (e != hipSuccess) return fail(ADMM_E_HIP, "%s: %s", #call, hipGetErrorString(e));   \
    } while (0)
    if (K == 0) {
        if (phases & 2) {
            if (y_bar) HIPCHK(hipMemsetAsync(y_bar, 0, planes * MN * 4, s));
            if (h_bar && kh > 0) HIPCHK(hipMemsetAsync(h_bar, 0, (size_t)kh * kw * 4, s));
            if (lambda_bar) HIPCHK(hipMemsetAsync(lambda_bar, 0, 4, s));
            if (rho_bar) HIPCHK(hipMemsetAsync(rho_bar, 0, 4, s));
        }
        if (phases & 1) HIPCHK(hipMemsetAsync(x_out, 0, planes * MN * 4, s));
        return ln.finish();
    }
    // ---- forward with trajectory ----
    Traj tr;
    tr.s = reinterpret_cast<float*>(ws + bl.traj_s);
    tr.m = use_masks && !iso ? reinterpret_cast<unsigned*>(ws + bl.traj_s) : nullptr;
    tr.iso_lane = iso_lane;
    tr.v = want_h ? reinterpret_cast<float2*>(ws + bl.traj_v) : nullptr;
    tr.sig = want_h ? reinterpret_cast<double2*>(ws + bl.sig) : nullptr;
    tr.nrm = iso ? reinterpret_cast<float*>(ws + bl.traj_n) : nullptr;
    if (phases & 1) {
        rc = run_forward(ln, y, xK, M, N, planes, h, kh, kw, sc, iso, K, ws, bl.f, tr, red, plan.fwd);
        if (rc) return rc;
    }
    if (!(phases & 2)) return ln.finish();
    // replay (phase 2 alone): the recording's {tau, rho, lambda} block is still in the workspace and is
    // used as is -- the reverse sweep must differentiate the trajectory that was recorded, even if a
    // device-resident lambda / rho has changed since (host values were checked against the tag above)
    // ---- reverse sweep ----
    float2* twM = reinterpret_cast<float2*>(ws + bl.f.twM);
    float2* twN = reinterpret_cast<float2*>(ws + bl.f.twN);
    float* Ct = reinterpret_cast<float*>(ws + bl.f.C);
    float2* Gt = kh > 0 ? reinterpret_cast<float2*>(ws + bl.f.G) : nullptr;
    float2* specA = reinterpret_cast<float2*>(ws + bl.f.spec0);
    float2* specB = reinterpret_cast<float2*>(ws + bl.f.spec1);
    float* sb[2] = {reinterpret_cast<float*>(ws + bl.sbA), reinterpret_cast<float*>(ws + bl.sbB)};
    // Vsum = sum_k vbar_k feeds y_bar and the h_bar correlation only: without either the sweep skips it
    const bool want_v = y_bar != nullptr || (h_bar != nullptr && kh > 0);
    float* vsum = want_v ? reinterpret_cast<float*>(ws + bl.vsum) : nullptr;
    // s_k and D x_K enter rho_bar's <D vbar, D x_k> only (fused and iso sweeps skip them without rho_bar)
    const bool want_rho = rho_bar != nullptr;
    double* rpart = reinterpret_cast<double*>(ws + bl.rpart);
    double* Qp = want_h ? reinterpret_cast<double*>(ws + bl.Qp) : nullptr;
    const size_t sstride = planes * 2 * MN;
    const size_t clds = column_lds(N, KB), flds = fwdinv_lds(M, T);
    const size_t alds = line_lds(M, T) + 8 * 16;
    const dim3 gl(N / T, (unsigned)planes), gc(L / KB, (unsigned)planes);
    // fused reverse sweep: one workgroup per plane runs all K steps (plane256_adj_kernel)
    const bool fused_adj = plan.bwd == ADMM_PATH_SWEEP_FUSED;
    int red_rows = K * bl.nblk_line;   // rows of (rho_bar, tau_bar) partials
    if (fused_adj) {
        namespace pk = admm::plane;
        float4* dxK = want_rho ? reinterpret_cast<float4*>(sb[1]) : nullptr;
        float* vout = !want_v ? nullptr : kh > 0 ? vsum : y_bar;
        if (want_rho) {
            rc = ln.run(ADMM_K_PREP, [&] { return pk::launch_dx_lane(xK, dxK, planes, s); });
            if (rc) return rc;
        }
        rc = ln.run(ADMM_K_ADJ, [&] {
            return pk::launch_plane_adj(x_bar, ws + bl.f.F, tr.m ? static_cast<const void*>(tr.m) : tr.s, dxK,
                                       reinterpret_cast<float4*>(sb[0]), specA, vout, rpart, prm, K, planes, s,
                                       nullptr, tr.m != nullptr);
        });
        if (rc) return rc;
        red_rows = (int)planes;
    } else if (iso_lane) {
        // isotropic fused sweep: per step one plane256_isoadj_kernel (B phase of step k+1, column phase, A phase
        // of step k) and one iso_radj_kernel (R_k over the batch, tau_bar rows); rows of step k at (K - k) x 512
        namespace pk = admm::plane;
        const size_t kE = MN / 2;   // lane-native float2 elements per plane
        float4* trs = reinterpret_cast<float4*>(tr.s);
        const float2* trn = reinterpret_cast<const float2*>(tr.nrm);
        float2* vbuf = reinterpret_cast<float2*>(ws + bl.wbar);
        float2* rmap = reinterpret_cast<float2*>(ws + bl.Rmap);
        float2* rpl = specB;    // per plane R partials (the forward's q partials, free now)
        float2* vsl = specA;    // lane-native Vsum (the forward's H^T y, free now)
        float* vout = !want_v ? nullptr : kh > 0 ? vsum : y_bar;
        HIPCHK(hipMemsetAsync(rpart, 0, (size_t)(K > 1 ? K - 1 : 1) * 512 * 2 * 8, s));
        for (int k = K; k >= 1; --k) {
            rc = ln.run(ADMM_K_ADJ, [&] {
                return pk::launch_plane_isoadj(x_bar, ws + bl.f.F, trs, planes * kE, trn, kE, vbuf,
                                               reinterpret_cast<float4*>(sb[0]), rmap, rpl, vsl, vout, prm, k, K, planes, s);
            });
            if (rc) return rc;
            if (k >= 2) {
                rc = ln.run(ADMM_K_NORM, [&] {
                    return pk::launch_iso_radj(rpl, rmap, trn + (size_t)(k - 2) * kE, rpart + (size_t)(K - k) * 512 * 2, 0,
                                               prm, planes, s);
                });
                if (rc) return rc;
                // sharded batch: tau_bar above used this shard's R (shard contributions add up); sbar needs the
                // whole batch's R
                if (red) {
                    rc = call_reducer(red, reinterpret_cast<float*>(rmap), MN, s);
                    if (rc) return rc;
                }
            }
        }
        red_rows = (K > 1 ? K - 1 : 1) * 512;
    } else if (want_v) {
        HIPCHK(hipMemsetAsync(vsum, 0, planes * MN * 4, s));
    }
    float* wbar = iso ? reinterpret_cast<float*>(ws + bl.wbar) : nullptr;
    float* Rmap = iso ? reinterpret_cast<float*>(ws + bl.Rmap) : nullptr;
    float* Rpart = iso ? reinterpret_cast<float*>(ws + bl.Rpart) : nullptr;
    const int ngi = iso_ngroups(planes);
    // k = 1 launches no ISO_ADJ_R: its partial rows must read as zero
    if (iso && !iso_lane) HIPCHK(hipMemsetAsync(rpart, 0, (size_t)K * bl.nblk_line * 2 * 8, s));
    if (Qp) HIPCHK(hipMemsetAsync(Qp, 0, planes * (size_t)(L + 1) * N * 8, s));
    if (gen) {
        // ---- runtime-length reverse sweep (admm_generic_bwd.hip): column, line inverse -> vbar_k in
        // HBM, then the line adjoint (aniso) or ISO_ADJ_A -> ISO_ADJ_R -> ISO_ADJ_B ----
        namespace g = admm::gen;
        const int H = M / 2 + 1;
        const g::FPlan pM = make_fplan(M), pN = make_fplan(N);
        const dim3 ggl(gen_nb(N, T), (unsigned)planes), ggc((H + KB - 1) / KB, (unsigned)planes);
        const size_t lfw = gen_lds_line(M, T, false), lup = gen_lds_line(M, T, true);
        const size_t lcol = gen_lds_col(N, KB);
        set_lds(g::line_fwd_kernel, lfw);
        set_lds(g::line_inv_kernel, lfw);
        set_lds(g::line_adj_kernel, lup);
        set_lds(g::iso_adj_b_kernel, lup);
        set_lds(g::column_kernel, lcol);
        float* vb = reinterpret_cast<float*>(ws + bl.f.xg);
        rc = ln.run(ADMM_K_PREP, [&] { hipLaunchKernelGGL(g::line_fwd_kernel, ggl, dim3(256), lfw, s, x_bar, specA, twM, pM, N, T); });
        if (rc) return rc;
        for (int k = K; k >= 1; --k) {
            float2* vs = want_h ? tr.v + (size_t)(k - 1) * planes * N * H : nullptr;
            rc = ln.run(ADMM_K_COLUMN, [&] {
                hipLaunchKernelGGL(g::column_kernel, ggc, dim3(256), lcol, s, specA, specB, Ct, Gt, twN, pN, H, KB,
                                   want_h ? 8 : 0, 1.0f, vs, Qp);
            });
            if (rc) return rc;
            rc = ln.run(ADMM_K_LINE, [&] { hipLaunchKernelGGL(g::line_inv_kernel, ggl, dim3(256), lfw, s, specB, vb, twM, pM, N, T); });
            if (rc) return rc;
            const float* sk1 = k >= 2 ? tr.s + (size_t)(k - 2) * sstride : nullptr;
            const float* skk = k < K ? tr.s + (size_t)(k - 1) * sstride : nullptr;
            const float* sbi = k < K ? sb[k & 1] : nullptr;
            float* sbo = sb[(k & 1) ^ 1];
            double* rp = rpart + (size_t)(K - k) * bl.nblk_line * 2;
            if (!iso) {
                rc = ln.run(ADMM_K_ADJ, [&] {
                    hipLaunchKernelGGL(g::line_adj_kernel, ggl, dim3(256), lup, s, vb, sk1, skk, xK, sbi, sbo, vsum, specA,
                                       rp, twM, pM, N, T, prm);
                });
                if (rc) return rc;
                continue;
            }
            const float* nrm1 = k >= 2 ? tr.nrm + (size_t)(k - 2) * MN : nullptr;
            rc = ln.run(ADMM_K_ADJ, [&] {
                hipLaunchKernelGGL(g::iso_adj_a_kernel, dim3(gen_nb(N, T), (unsigned)ngi), dim3(256), (size_t)T * M * 4, s, vb,
                                   sk1, skk, xK, nrm1, sbi, wbar, vsum, Rpart, rp, M, N, (int)planes, iso_group(planes),
                                   T, prm);
            });
            if (rc) return rc;
            if (k == 1) break;
            rc = ln.run(ADMM_K_NORM, [&] {
                hipLaunchKernelGGL(admm::iso_adj_r_kernel, dim3(kIsoAdjRBlocks), dim3(kThreads), 0, s, Rpart, Rmap,
                                   nrm1, ngi, MN, prm, rp + (size_t)bl.nblk_isoA * 2);
            });
            if (rc) return rc;
            if (red) {
                rc = call_reducer(red, Rmap, MN, s);
                if (rc) return rc;
            }
            rc = ln.run(ADMM_K_ADJ, [&] {
                hipLaunchKernelGGL(g::iso_adj_b_kernel, ggl, dim3(256), lup, s, wbar, sbi, sk1, nrm1, Rmap, sbo, specA,
                                   twM, pM, N, T, prm);
            });
            if (rc) return rc;
        }
    } else if (!fused_adj && !iso_lane) {
        rc = ln.run(ADMM_K_PREP, [&] { return launch_line_fwd(L, T, gl, flds, s, x_bar, specA, twM, N); });
        if (rc) return rc;
    }
    for (int k = (fused_adj || gen || iso_lane) ? 0 : K; k >= 1; --k) {
        float2* vs = want_h ? tr.v + (size_t)(k - 1) * planes * N * L : nullptr;
        rc = ln.run(ADMM_K_COLUMN, [&] {
            return launch_column(N, want_h ? 4 : 0, gc, clds, s, specA, specB, Ct, Gt, twN, L, KB, 1.0f, vs, Qp);
        });
        if (rc) return rc;
        const float* sk1 = k >= 2 ? tr.s + (size_t)(k - 2) * sstride : nullptr;
        const float* skk = k < K ? tr.s + (size_t)(k - 1) * sstride : nullptr;
        const float* sbi = k < K ? sb[k & 1] : nullptr;
        float* sbo = sb[(k & 1) ^ 1];
        double* rp = rpart + (size_t)(K - k) * bl.nblk_line * 2;
        if (!iso) {
            rc = ln.run(ADMM_K_ADJ, [&] {
                return launch_line_adj(L, T, gl, alds, s, specB, sk1, want_rho ? skk : nullptr, want_rho ? xK : nullptr,
                                       sbi, sbo, vsum, specA, rp, twM, N, prm,
                                k == 1 ? 1 : 0, k == K ? 1 : 0, ln_traj);
            });
            if (rc) return rc;
            continue;
        }
        // isotropic: ISO_ADJ_A (plane groups) -> ISO_ADJ_R (batch R map, tau_bar) -> ISO_ADJ_B (per plane)
        const float* nrm1 = k >= 2 ? tr.nrm + (size_t)(k - 2) * MN : nullptr;
        rc = ln.run(ADMM_K_ADJ, [&] {
            return launch_iso_adj_a(L, T, dim3(N / T, (unsigned)ngi), iso_a_lds(M, T) + 8 * 16, s, specB, sk1,
                             want_rho ? skk : nullptr, want_rho ? xK : nullptr,
                             nrm1, sbi, wbar, vsum, Rpart, rp, twM, N, (int)planes, iso_group(planes), prm,
                             k == 1 ? 1 : 0, k == K ? 1 : 0);
        });
        if (rc) return rc;
        if (k == 1) break;
        rc = ln.run(ADMM_K_NORM, [&] {
            hipLaunchKernelGGL(admm::iso_adj_r_kernel, dim3(kIsoAdjRBlocks), dim3(kThreads), 0, s, Rpart, Rmap, nrm1,
                               ngi, MN, prm, rp + (size_t)bl.nblk_isoA * 2);
        });
        if (rc) return rc;
        // sharded batch: tau_bar above used this shard's R (shard contributions add up, like every other
        // parameter gradient); sbar needs the whole batch's R
        if (red) {
            rc = call_reducer(red, Rmap, MN, s);
            if (rc) return rc;
        }
        rc = ln.run(ADMM_K_ADJ, [&] {
            return launch_iso_adj_b(L, T, gl, iso_b_lds(M, T), s, wbar, sbi, sk1, nrm1, Rmap, sbo, specA, twM, N, prm);
        });
        if (rc) return rc;
    }
    // ---- assembly ----
    double* rt = reinterpret_cast<double*>(ws + bl.rt);
    rc = ln.run(ADMM_K_FINAL, [&] {
        launch_reduce_cols(s, rpart, rt, red_rows, 2, reinterpret_cast<double*>(ws + bl.rtmp));
    });
    if (rc) return rc;
    double* hcorr = kh > 0 ? reinterpret_cast<double*>(ws + bl.hcorr) : nullptr;
    double* hA = want_h ? reinterpret_cast<double*>(ws + bl.hA) : nullptr;
    if (kh > 0 && want_v) {
        // y_bar = H vsum  (centred circular convolution, spectrally)
        if (y_bar && gen) {
            namespace g = admm::gen;
            const int H = M / 2 + 1;
            const g::FPlan pM = make_fplan(M), pN = make_fplan(N);
            const dim3 ggl(gen_nb(N, T), (unsigned)planes), ggc((H + KB - 1) / KB, (unsigned)planes);
            const size_t lfw = gen_lds_line(M, T, false), lcol = gen_lds_col(N, KB);
            rc = ln.run(ADMM_K_FINAL, [&] { hipLaunchKernelGGL(g::line_fwd_kernel, ggl, dim3(256), lfw, s, vsum, specA, twM, pM, N, T); });
            if (rc) return rc;
            rc = ln.run(ADMM_K_FINAL, [&] {
                hipLaunchKernelGGL(g::column_kernel, ggc, dim3(256), lcol, s, specA, specB, Ct, Gt, twN, pN, H, KB, 2, 1.0f,
                                   (float2*)nullptr, (double*)nullptr);
            });
            if (rc) return rc;
            rc = ln.run(ADMM_K_FINAL, [&] { hipLaunchKernelGGL(g::line_inv_kernel, ggl, dim3(256), lfw, s, specB, y_bar, twM, pM, N, T); });
            if (rc) return rc;
        } else if (y_bar) {
            rc = ln.run(ADMM_K_FINAL, [&] { return launch_line_fwd(L, T, gl, flds, s, vsum, specA, twM, N); });
            if (rc) return rc;
            rc = ln.run(ADMM_K_FINAL, [&] { return launch_column(N, 2, gc, clds, s, specA, specB, Ct, Gt, twN, L, KB, 1.0f); });
            if (rc) return rc;
            rc = ln.run(ADMM_K_FINAL, [&] { return launch_line_inv(L, T, gl, flds, s, specB, y_bar, twM, N); });
            if (rc) return rc;
        }
        if (h_bar) {
            double* hpart = reinterpret_cast<double*>(ws + bl.hpart);
            rc = ln.run(ADMM_K_FINAL, [&] {
                const size_t lds = (size_t)(2 * bl.TY + kw - 1) * M * 4;
                set_lds(admm::hbar_corr_kernel, lds);
                hipLaunchKernelGGL(admm::hbar_corr_kernel, dim3(N / bl.TY, (unsigned)planes), dim3(kThreads), lds, s,
                                   vsum, y, hpart, M, N, kh, kw, bl.TY);
            });
            if (rc) return rc;
            rc = ln.run(ADMM_K_FINAL, [&] {
                launch_reduce_cols(s, hpart, hcorr, bl.nblk_corr, kh * kw, reinterpret_cast<double*>(ws + bl.rtmp));
            });
            if (rc) return rc;
            double* Q = reinterpret_cast<double*>(ws + bl.Q);
            const int nq = (L + 1) * N;
            rc = ln.run(ADMM_K_FINAL, [&] {
                hipLaunchKernelGGL(admm::reduce_planes_kernel, dim3((nq + 255) / 256), dim3(256), 0, s, Qp, Q,
                                   (int)planes, nq);
            });
            if (rc) return rc;
            rc = ln.run(ADMM_K_FINAL, [&] {
                hipLaunchKernelGGL(admm::hbarA_kernel, dim3(kh * kw), dim3(kThreads), 0, s, Q, Ct, tr.sig, kh, M, N,
                                   hA);
            });
            if (rc) return rc;
        }
    } else if (!fused_adj && !iso_lane && y_bar) {   // (the fused sweeps wrote Vsum straight into y_bar)
        HIPCHK(hipMemcpyAsync(y_bar, vsum, planes * MN * 4, hipMemcpyDeviceToDevice, s));
    }
    rc = ln.run(ADMM_K_FINAL, [&] {
        const int nt = kh * kw > 1 ? kh * kw : 1;
        hipLaunchKernelGGL(admm::grads_final_kernel, dim3((nt + 255) / 256), dim3(256), 0, s, rt, hcorr, hA, kh * kw,
                           prm, lambda_bar, rho_bar, (h_bar && kh > 0) ? h_bar : nullptr);
    });
    if (rc) return rc;
#undef HIPCHK
    return ln.finish();
}

// ---- several branches below the plane-count rule: the 2-pass kernels over every branch's planes ----
// Grid plane q = i ppb + loc is branch i's solve of input plane loc (y shared, x_out / x_bar in the chcat layout:
// the line transforms map planes, admm_kernels.hip PlaneMap); per branch its C table, {tau, rho, lambda}, f map,
// |s| slots, R map and plane groups.  The step sequences are run_forward's / launch_backward's 2-pass ones.
Branches multi2_branches(int P, int B, int nbr) { return Branches{P * B, nbr, P, (unsigned)(multi_C_bytes() / 4), 4u}; }

int run_multi_2pass_iso_fwd(Launcher& ln, const float* y, float* x_out, int P, int B, int nbr, int maxit, bool rec,
                            unsigned char* ws, size_t planes, const MultiLayout& Ly) {
    hipStream_t s = ln.s;
    constexpr int M = kMultiM, N = kMultiN, L = M / 2;
    const size_t MN = (size_t)M * N, ppb = (size_t)P * B, sstride = planes * 2 * MN;
    const Branches br = multi2_branches(P, B, nbr);
    const int T = line_T(M, N), KB = column_KB(M, N);
    const size_t flds = fwdinv_lds(M, T), clds = column_lds(N, KB);
    const dim3 gl(N / T, (unsigned)planes), gc(L / KB, (unsigned)planes);
    float2* twM = reinterpret_cast<float2*>(ws + Ly.twM);
    float2* twN = reinterpret_cast<float2*>(ws + Ly.twN);
    const float* Ct = reinterpret_cast<const float*>(ws + Ly.C);
    const float* prm = reinterpret_cast<const float*>(ws + Ly.prm);
    float2* spec0 = reinterpret_cast<float2*>(ws + Ly.spec0);
    float2* spec1 = reinterpret_cast<float2*>(ws + Ly.spec1);
    float* fmap = reinterpret_cast<float*>(ws + Ly.fmap);
    float* qpart = reinterpret_cast<float*>(ws + Ly.qpart);
    float* traj = rec ? reinterpret_cast<float*>(ws + Ly.traj) : nullptr;
    float* nrm = rec ? reinterpret_cast<float*>(ws + Ly.nrm) : nullptr;
    float* sA = rec ? nullptr : reinterpret_cast<float*>(ws + Ly.sA);
    // H^T y = y (no PSF) in the spectral domain, as run_forward's 2-pass kernels: Y_h = F y per grid plane (the
    // hln slot, unused by the 2-pass grid), added by every column pass; iteration 1 transforms a zero spectrum
    float2* yh = reinterpret_cast<float2*>(ws + Ly.hln);
    int rc = ln.run(ADMM_K_PREP, [&] { return launch_line_fwd(L, T, gl, flds, s, y, spec0, twM, N, br, kMapIn); });
    if (rc) return rc;
    rc = ln.run(ADMM_K_PREP, [&] {
        return launch_column(N, 5, gc, clds, s, spec0, spec1, Ct, nullptr, twN, L, KB, 1.0f, nullptr, nullptr, br, yh);
    });
    if (rc) return rc;
    if (hipMemsetAsync(spec0, 0, planes * MN * 4, s) != hipSuccess) return fail(ADMM_E_HIP, "hipMemsetAsync");
    for (int it = 1; it <= maxit; ++it) {
        rc = ln.run(ADMM_K_COLUMN, [&] {
            return launch_column(N, 6, gc, clds, s, spec0, spec1, Ct, nullptr, twN, L, KB, 1.0f, nullptr, nullptr, br, yh);
        });
        if (rc) return rc;
        if (it == maxit) {
            rc = ln.run(ADMM_K_FINAL, [&] { return launch_line_inv(L, T, gl, flds, s, spec1, x_out, twM, N, br, kMapOut); });
            if (rc) return rc;
            break;
        }
        // recording: s_it into slot it - 1 (the first iteration reads no s), |s_it| into norm slot it - 1
        float* sn = rec ? traj + (size_t)(it - 1) * sstride : sA;
        const float* so = rec ? (it >= 2 ? traj + (size_t)(it - 2) * sstride : sn) : sA;
        float* nrm_out = rec ? nrm + (size_t)(it - 1) * nbr * MN : nullptr;
        rc = ln.run(ADMM_K_LINE, [&] {
            return launch_iso_a(L, T, dim3(N / T, (unsigned)(nbr * Ly.ngb)), iso_a_lds(M, T), s, spec1, so, sn, fmap,
                                qpart, twM, N, (int)ppb, Ly.G, it == 1 ? 1 : 0, Ly.ngb);
        });
        if (rc) return rc;
        rc = ln.run(ADMM_K_NORM, [&] {
            hipLaunchKernelGGL(admm::iso_r_kernel, dim3((unsigned)std::min<size_t>((MN + 63) / 64, 2048), (unsigned)nbr),
                               dim3(kThreads), 0, s, qpart, fmap, Ly.ngb, MN, prm, nrm_out, 4u);
        });
        if (rc) return rc;
        rc = ln.run(ADMM_K_LINE, [&] {
            return launch_iso_b(L, T, gl, iso_b_lds(M, T), s, sn, fmap, nullptr, spec0, twM, N, prm, br);
        });
        if (rc) return rc;
    }
    return ADMM_OK;
}

int run_multi_2pass_iso_bwd(Launcher& ln, const float* x_bar, float* y_bar, float* lambda_bar, int P, int B, int nbr,
                            int K, unsigned char* ws, size_t planes, const MultiLayout& Ly) {
    hipStream_t s = ln.s;
    constexpr int M = kMultiM, N = kMultiN, L = M / 2;
    const size_t MN = (size_t)M * N, ppb = (size_t)P * B, sstride = planes * 2 * MN;
    const Branches br = multi2_branches(P, B, nbr);
    const int T = bwd_line_T(M, N, true), KB = column_KB(M, N);
    const size_t flds = fwdinv_lds(M, T), clds = column_lds(N, KB);
    const dim3 gl(N / T, (unsigned)planes), gc(L / KB, (unsigned)planes);
    float2* twM = reinterpret_cast<float2*>(ws + Ly.twM);
    float2* twN = reinterpret_cast<float2*>(ws + Ly.twN);
    const float* Ct = reinterpret_cast<const float*>(ws + Ly.C);
    const float* prm = reinterpret_cast<const float*>(ws + Ly.prm);
    float2* specA = reinterpret_cast<float2*>(ws + Ly.spec0);
    float2* specB = reinterpret_cast<float2*>(ws + Ly.spec1);
    const float* traj = reinterpret_cast<const float*>(ws + Ly.traj);
    const float* nrm = reinterpret_cast<const float*>(ws + Ly.nrm);
    float* sb[2] = {reinterpret_cast<float*>(ws + Ly.sbA), reinterpret_cast<float*>(ws + Ly.sbB)};
    float* vsum = y_bar ? reinterpret_cast<float*>(ws + Ly.vsum) : nullptr;
    float* wbar = reinterpret_cast<float*>(ws + Ly.wbar);
    float* Rmap = reinterpret_cast<float*>(ws + Ly.rmap);
    float* Rpart = reinterpret_cast<float*>(ws + Ly.Rpart);
    double* part = reinterpret_cast<double*>(ws + Ly.part);
    hipError_t e = hipMemsetAsync(part, 0, (size_t)nbr * Ly.pbs * 8, s);   // k = 1 launches no ISO_ADJ_R
    if (e == hipSuccess && vsum) e = hipMemsetAsync(vsum, 0, planes * MN * 4, s);
    if (e != hipSuccess) return fail(ADMM_E_HIP, "hipMemsetAsync: %s", hipGetErrorString(e));
    int rc = ln.run(ADMM_K_PREP, [&] { return launch_line_fwd(L, T, gl, flds, s, x_bar, specA, twM, N, br, kMapOut); });
    if (rc) return rc;
    for (int k = K; k >= 1; --k) {
        rc = ln.run(ADMM_K_COLUMN, [&] {
            return launch_column(N, 0, gc, clds, s, specA, specB, Ct, nullptr, twN, L, KB, 1.0f, nullptr, nullptr, br);
        });
        if (rc) return rc;
        const float* sk1 = k >= 2 ? traj + (size_t)(k - 2) * sstride : nullptr;
        const float* sbi = k < K ? sb[k & 1] : nullptr;
        float* sbo = sb[(k & 1) ^ 1];
        double* rp = part + (size_t)(K - k) * Ly.rows_b * 2;
        const float* nrm1 = k >= 2 ? nrm + (size_t)(k - 2) * nbr * MN : nullptr;
        rc = ln.run(ADMM_K_ADJ, [&] {
            return launch_iso_adj_a(L, T, dim3(N / T, (unsigned)(nbr * Ly.ngb)), iso_a_lds(M, T) + 8 * 16, s, specB, sk1,
                                    nullptr, nullptr, nrm1, sbi, wbar, vsum, Rpart, rp, twM, N, (int)ppb, Ly.G, prm,
                                    k == 1 ? 1 : 0, k == K ? 1 : 0, br, Ly.ngb, Ly.pbs);
        });
        if (rc) return rc;
        if (k == 1) break;
        rc = ln.run(ADMM_K_NORM, [&] {
            hipLaunchKernelGGL(admm::iso_adj_r_kernel, dim3(kIsoAdjRBlocks, (unsigned)nbr), dim3(kThreads), 0, s, Rpart,
                               Rmap, nrm1, Ly.ngb, MN, prm, rp + (size_t)Ly.nblk_a * 2, 4u, Ly.pbs);
        });
        if (rc) return rc;
        rc = ln.run(ADMM_K_ADJ, [&] {
            return launch_iso_adj_b(L, T, gl, iso_b_lds(M, T), s, wbar, sbi, sk1, nrm1, Rmap, sbo, specA, twM, N, prm, br);
        });
        if (rc) return rc;
    }
    double* rt = reinterpret_cast<double*>(ws + Ly.rt);
    for (int i = 0; i < nbr; ++i) {
        rc = ln.run(ADMM_K_FINAL, [&] {
            launch_reduce_cols(s, part + (size_t)i * Ly.pbs, rt + 2 * i, K * Ly.rows_b, 2,
                               reinterpret_cast<double*>(ws + Ly.rtmp));
        });
        if (rc) return rc;
        rc = ln.run(ADMM_K_FINAL, [&] {
            hipLaunchKernelGGL(admm::grads_final_kernel, dim3(1), dim3(64), 0, s, rt + 2 * i, (const double*)nullptr,
                               (const double*)nullptr, 0, prm + 4 * i, lambda_bar ? lambda_bar + i : nullptr,
                               (float*)nullptr, (float*)nullptr);
        });
        if (rc) return rc;
    }
    if (y_bar) {
        rc = ln.run(ADMM_K_FINAL, [&] {
            hipLaunchKernelGGL(admm::branch_sum_kernel, dim3(1024), dim3(kThreads), 0, s, vsum, y_bar, ppb * MN, nbr);
        });
        if (rc) return rc;
    }
    return ADMM_OK;
}

int run_multi_2pass_fwd(Launcher& ln, const float* y, float* x_out, int P, int B, int nbr, int maxit, bool rec,
                        unsigned char* ws, size_t planes, const MultiLayout& Ly) {
    hipStream_t s = ln.s;
    constexpr int M = kMultiM, N = kMultiN, L = M / 2;
    const size_t MN = (size_t)M * N, sstride = planes * 2 * MN;
    const Branches br = multi2_branches(P, B, nbr);
    const int T = line_T(M, N), KB = column_KB(M, N);
    const size_t llds = line_lds(M, T), flds = fwdinv_lds(M, T), clds = column_lds(N, KB);
    const dim3 gl(N / T, (unsigned)planes), gc(L / KB, (unsigned)planes);
    float2* twM = reinterpret_cast<float2*>(ws + Ly.twM);
    float2* twN = reinterpret_cast<float2*>(ws + Ly.twN);
    const float* Ct = reinterpret_cast<const float*>(ws + Ly.C);
    const float* prm = reinterpret_cast<const float*>(ws + Ly.prm);
    float2* spec0 = reinterpret_cast<float2*>(ws + Ly.spec0);
    float2* spec1 = reinterpret_cast<float2*>(ws + Ly.spec1);
    float* traj = rec ? reinterpret_cast<float*>(ws + Ly.traj) : nullptr;
    float* sbuf[2] = {rec ? nullptr : reinterpret_cast<float*>(ws + Ly.sA), rec ? nullptr : reinterpret_cast<float*>(ws + Ly.sbA)};
    // H^T y = y (no PSF) in the spectral domain, as run_forward's 2-pass kernels: Y_h = F y per grid plane (the
    // hln slot, unused by the 2-pass grid), added by every column pass; iteration 1 transforms a zero spectrum
    float2* yh = reinterpret_cast<float2*>(ws + Ly.hln);
    int rc = ln.run(ADMM_K_PREP, [&] { return launch_line_fwd(L, T, gl, flds, s, y, spec0, twM, N, br, kMapIn); });
    if (rc) return rc;
    rc = ln.run(ADMM_K_PREP, [&] {
        return launch_column(N, 5, gc, clds, s, spec0, spec1, Ct, nullptr, twN, L, KB, 1.0f, nullptr, nullptr, br, yh);
    });
    if (rc) return rc;
    if (hipMemsetAsync(spec0, 0, planes * MN * 4, s) != hipSuccess) return fail(ADMM_E_HIP, "hipMemsetAsync");
    for (int it = 1; it <= maxit; ++it) {
        rc = ln.run(ADMM_K_COLUMN, [&] {
            return launch_column(N, 6, gc, clds, s, spec0, spec1, Ct, nullptr, twN, L, KB, 1.0f, nullptr, nullptr, br, yh);
        });
        if (rc) return rc;
        if (it == maxit) {
            rc = ln.run(ADMM_K_FINAL, [&] { return launch_line_inv(L, T, gl, flds, s, spec1, x_out, twM, N, br, kMapOut); });
            if (rc) return rc;
            break;
        }
        // recording: s_it into slot it - 1 (the first iteration reads no s); otherwise the two s buffers in turn
        float* sn = rec ? traj + (size_t)(it - 1) * sstride : ((it & 1) ? sbuf[0] : sbuf[1]);
        const float* so = rec ? (it >= 2 ? traj + (size_t)(it - 2) * sstride : sn) : ((it & 1) ? sbuf[1] : sbuf[0]);
        rc = ln.run(ADMM_K_LINE, [&] {
            return launch_line(L, T, gl, llds, s, spec1, spec0, so, sn, nullptr, twM, N, prm, it == 1 ? 1 : 0, kThreads, br);
        });
        if (rc) return rc;
    }
    return ADMM_OK;
}

int run_multi_2pass_bwd(Launcher& ln, const float* x_bar, float* y_bar, float* lambda_bar, float* rho_bar,
                        const float* x_out, int P, int B, int nbr, int K, unsigned char* ws, size_t planes,
                        const MultiLayout& Ly) {
    hipStream_t s = ln.s;
    constexpr int M = kMultiM, N = kMultiN, L = M / 2;
    const size_t MN = (size_t)M * N, ppb = (size_t)P * B, sstride = planes * 2 * MN;
    const Branches br = multi2_branches(P, B, nbr);
    const int T = bwd_line_T(M, N, false), KB = column_KB(M, N);
    const size_t alds = line_lds(M, T) + 8 * 16, flds = fwdinv_lds(M, T), clds = column_lds(N, KB);
    const dim3 gl(N / T, (unsigned)planes), gc(L / KB, (unsigned)planes);
    float2* twM = reinterpret_cast<float2*>(ws + Ly.twM);
    float2* twN = reinterpret_cast<float2*>(ws + Ly.twN);
    const float* Ct = reinterpret_cast<const float*>(ws + Ly.C);
    const float* prm = reinterpret_cast<const float*>(ws + Ly.prm);
    float2* specA = reinterpret_cast<float2*>(ws + Ly.spec0);
    float2* specB = reinterpret_cast<float2*>(ws + Ly.spec1);
    const float* traj = reinterpret_cast<const float*>(ws + Ly.traj);
    float* sb[2] = {reinterpret_cast<float*>(ws + Ly.sbA), reinterpret_cast<float*>(ws + Ly.sbB)};
    float* vsum = y_bar ? reinterpret_cast<float*>(ws + Ly.vsum) : nullptr;
    double* part = reinterpret_cast<double*>(ws + Ly.part);
    hipError_t e = vsum ? hipMemsetAsync(vsum, 0, planes * MN * 4, s) : hipSuccess;
    if (e != hipSuccess) return fail(ADMM_E_HIP, "hipMemsetAsync: %s", hipGetErrorString(e));
    int rc = ln.run(ADMM_K_PREP, [&] { return launch_line_fwd(L, T, gl, flds, s, x_bar, specA, twM, N, br, kMapOut); });
    if (rc) return rc;
    for (int k = K; k >= 1; --k) {
        rc = ln.run(ADMM_K_COLUMN, [&] {
            return launch_column(N, 0, gc, clds, s, specA, specB, Ct, nullptr, twN, L, KB, 1.0f, nullptr, nullptr, br);
        });
        if (rc) return rc;
        const float* sk1 = k >= 2 ? traj + (size_t)(k - 2) * sstride : nullptr;
        const float* skk = k < K ? traj + (size_t)(k - 1) * sstride : nullptr;
        const float* sbi = k < K ? sb[k & 1] : nullptr;
        float* sbo = sb[(k & 1) ^ 1];
        double* rp = part + (size_t)(K - k) * Ly.rows_b * 2;
        rc = ln.run(ADMM_K_ADJ, [&] {
            return launch_line_adj(L, T, gl, alds, s, specB, sk1, rho_bar ? skk : nullptr, rho_bar ? x_out : nullptr, sbi,
                                   sbo, vsum, specA, rp, twM, N, prm, k == 1 ? 1 : 0, k == K ? 1 : 0, false, br, Ly.pbs);
        });
        if (rc) return rc;
    }
    double* rt = reinterpret_cast<double*>(ws + Ly.rt);
    for (int i = 0; i < nbr; ++i) {
        rc = ln.run(ADMM_K_FINAL, [&] {
            launch_reduce_cols(s, part + (size_t)i * Ly.pbs, rt + 2 * i, K * Ly.rows_b, 2,
                               reinterpret_cast<double*>(ws + Ly.rtmp));
        });
        if (rc) return rc;
        rc = ln.run(ADMM_K_FINAL, [&] {
            hipLaunchKernelGGL(admm::grads_final_kernel, dim3(1), dim3(64), 0, s, rt + 2 * i, (const double*)nullptr,
                               (const double*)nullptr, 0, prm + 4 * i, lambda_bar ? lambda_bar + i : nullptr,
                               rho_bar ? rho_bar + i : nullptr, (float*)nullptr);
        });
        if (rc) return rc;
    }
    if (y_bar) {
        rc = ln.run(ADMM_K_FINAL, [&] {
            hipLaunchKernelGGL(admm::branch_sum_kernel, dim3(1024), dim3(kThreads), 0, s, vsum, y_bar, ppb * MN, nbr);
        });
        if (rc) return rc;
    }
    return ADMM_OK;
}

int launch_forward_multi(const float* y, float* x_out, int M, int N, int P, int B, int nbr, const float* const* lambda,
                         const float* const* rho, int maxit, int flags, void* workspace, void* stream, size_t planes,
                         const MultiLayout& L) {
    int rc = ADMM_OK;
    unsigned char* ws = static_cast<unsigned char*>(workspace);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    Launcher ln{s, g_prof.on, {}};
    float* prm = reinterpret_cast<float*>(ws + L.prm);
    float2* twM = reinterpret_cast<float2*>(ws + L.twM);
    float2* twN = reinterpret_cast<float2*>(ws + L.twN);
    for (int i = 0; i < nbr; ++i) {
        float* Ct = reinterpret_cast<float*>(ws + L.C + (size_t)i * multi_C_bytes());
        void* F = ws + L.F + (size_t)i * multi_F_bytes();
        const admm::ScalarSrc sc{lambda[i], rho[i], 0.f, 0.f};
        rc = ln.run(ADMM_K_SETUP, [&] {
            const size_t lds = (size_t)(M + N) * 16;
            const int nb = (int)(((size_t)(M / 2 + 1) * N + kThreads - 1) / kThreads);
            set_lds(admm::setup_kernel, lds);
            hipLaunchKernelGGL(admm::setup_kernel, dim3(nb < 1024 ? nb : 1024), dim3(kThreads), lds, s, twM, twN, Ct,
                               (float2*)nullptr, (const float*)nullptr, 0, 0, M, N, sc, prm + 4 * i, (double2*)nullptr);
        });
        if (rc) return rc;
        if (L.two_pass) continue;   // the 2-pass kernels read Ct itself
        rc = ln.run(ADMM_K_SETUP, [&] { return admm::plane::launch_tables(Ct, nullptr, F, s); });
        if (rc) return rc;
    }
    if (maxit == 0) {
        hipError_t e = hipMemsetAsync(x_out, 0, planes * (size_t)M * N * 4, s);
        if (e != hipSuccess) return fail(ADMM_E_HIP, "hipMemsetAsync: %s", hipGetErrorString(e));
        return ln.finish();
    }
    const bool rec = (flags & ADMM_MULTI_RECORD) != 0, masks = rec && (flags & ADMM_REC_MASKS) != 0;
    if (L.two_pass) {
        rc = (flags & ADMM_MULTI_ISO) ? run_multi_2pass_iso_fwd(ln, y, x_out, P, B, nbr, maxit, rec, ws, planes, L)
                                      : run_multi_2pass_fwd(ln, y, x_out, P, B, nbr, maxit, rec, ws, planes, L);
        if (rc) return rc;
        return ln.finish();
    }
    const admm::plane::Branches br = multi_branches(P, B, nbr);
    if (flags & ADMM_MULTI_ISO) {
        // isotropic: per iteration one plane256_iso_kernel over every branch's planes and one iso_norm_kernel
        // (each branch's batch norm over its own planes); recording: s_{k+1} into slot k, |s_{k+1}| too
        namespace pk = admm::plane;
        const size_t kE = (size_t)M * N / 2;
        float4* st = reinterpret_cast<float4*>(ws + (rec ? L.traj : L.sln));
        const size_t tslot = rec ? planes * kE : 0;
        float2* fl = reinterpret_cast<float2*>(ws + L.fmap);
        float2* ql = reinterpret_cast<float2*>(ws + L.qpart);
        for (int k = 0; k < maxit; ++k) {
            rc = ln.run(ADMM_K_PLANE, [&] {
                return pk::launch_plane_iso(y, x_out, ws + L.F, false, reinterpret_cast<float2*>(ws + L.hln),
                                            st + (k > 0 ? (size_t)(k - 1) * tslot : 0), st + (size_t)k * tslot, fl, ql,
                                            prm, k, maxit, planes, s, &br);
            });
            if (rc) return rc;
            if (k + 1 < maxit) {
                float2* nr = rec ? reinterpret_cast<float2*>(ws + L.nrm) + (size_t)k * nbr * kE : nullptr;
                rc = ln.run(ADMM_K_NORM, [&] { return pk::launch_iso_norm(ql, fl, nr, prm, planes, s, &br); });
                if (rc) return rc;
            }
        }
        return ln.finish();
    }
    rc = ln.run(ADMM_K_PLANE, [&] {
        return admm::plane::launch_plane(y, x_out, ws + L.F, false, reinterpret_cast<float2*>(ws + L.hln),
                                         reinterpret_cast<float4*>(ws + L.sln), prm, maxit, planes, s,
                                         rec && !masks ? reinterpret_cast<float4*>(ws + L.traj) : nullptr, &br,
                                         masks ? reinterpret_cast<unsigned*>(ws + L.traj) : nullptr);
    });
    if (rc) return rc;
    return ln.finish();
}

int launch_backward_multi(const float* x_bar, float* y_bar, float* lambda_bar, float* rho_bar, int M, int N, int P,
                          int B, int nbr, int maxit, const float* x_out, void* workspace, void* stream, int flags,
                          size_t planes, size_t ppb, size_t MN, const MultiLayout& L) {
    int rc = ADMM_OK;
    unsigned char* ws = static_cast<unsigned char*>(workspace);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    Launcher ln{s, g_prof.on, {}};
    hipError_t e;
    const int K = maxit;
    if (K == 0) {
        if (y_bar && (e = hipMemsetAsync(y_bar, 0, ppb * MN * 4, s)) != hipSuccess) return fail(ADMM_E_HIP, "memset");
        if (lambda_bar && (e = hipMemsetAsync(lambda_bar, 0, (size_t)nbr * 4, s)) != hipSuccess) return fail(ADMM_E_HIP, "memset");
        if (rho_bar && (e = hipMemsetAsync(rho_bar, 0, (size_t)nbr * 4, s)) != hipSuccess) return fail(ADMM_E_HIP, "memset");
        return ln.finish();
    }
    if (L.two_pass) {
        rc = (flags & ADMM_MULTI_ISO)
                 ? run_multi_2pass_iso_bwd(ln, x_bar, y_bar, lambda_bar, P, B, nbr, K, ws, planes, L)
                 : run_multi_2pass_bwd(ln, x_bar, y_bar, lambda_bar, rho_bar, x_out, P, B, nbr, K, ws, planes, L);
        if (rc) return rc;
        return ln.finish();
    }
    const admm::plane::Branches br = multi_branches(P, B, nbr);
    const float* prm = reinterpret_cast<const float*>(ws + L.prm);
    const bool masks = (flags & ADMM_REC_MASKS) != 0;
    if (flags & ADMM_MULTI_ISO) {
        // isotropic fused sweep over every branch's planes (plane_iso.hip): per reverse step one
        // plane256_isoadj_kernel and one iso_radj_kernel; vbar in the forward's dead s state, Vsum lane-native
        // in vsl and natural (per grid plane) in the H^T y slots, R partials in the q partial slots
        namespace pk = admm::plane;
        const size_t kE = MN / 2, rows = multi_iso_rows(K);
        float4* trs = reinterpret_cast<float4*>(ws + L.traj);
        const float2* trn = reinterpret_cast<const float2*>(ws + L.nrm);
        float2* vb = reinterpret_cast<float2*>(ws + L.sln);
        float2* rmap = reinterpret_cast<float2*>(ws + L.rmap);
        float2* rpl = reinterpret_cast<float2*>(ws + L.qpart);
        float* vout = y_bar ? reinterpret_cast<float*>(ws + L.hln) : nullptr;
        double* part = reinterpret_cast<double*>(ws + L.part);
        if ((e = hipMemsetAsync(part, 0, (size_t)nbr * rows * 16, s)) != hipSuccess) return fail(ADMM_E_HIP, "memset");
        for (int k = K; k >= 1; --k) {
            rc = ln.run(ADMM_K_ADJ, [&] {
                return pk::launch_plane_isoadj(x_bar, ws + L.F, trs, planes * kE, trn, nbr * kE, vb,
                                               reinterpret_cast<float4*>(ws + L.sbar), rmap, rpl,
                                               reinterpret_cast<float2*>(ws + L.vsl), vout, prm, k, K, planes, s, &br);
            });
            if (rc) return rc;
            if (k >= 2) {
                rc = ln.run(ADMM_K_NORM, [&] {
                    return pk::launch_iso_radj(rpl, rmap, trn + (size_t)(k - 2) * nbr * kE,
                                               part + (size_t)(K - k) * 512 * 2, rows * 2, prm, planes, s, &br);
                });
                if (rc) return rc;
            }
        }
        double* rt = reinterpret_cast<double*>(ws + L.rt);
        for (int i = 0; i < nbr; ++i) {
            rc = ln.run(ADMM_K_FINAL, [&] {
                launch_reduce_cols(s, part + (size_t)i * rows * 2, rt + 2 * i, (int)rows, 2,
                                   reinterpret_cast<double*>(ws + L.rtmp));
            });
            if (rc) return rc;
            rc = ln.run(ADMM_K_FINAL, [&] {
                hipLaunchKernelGGL(admm::grads_final_kernel, dim3(1), dim3(64), 0, s, rt + 2 * i, (const double*)nullptr,
                                   (const double*)nullptr, 0, prm + 4 * i, lambda_bar ? lambda_bar + i : nullptr,
                                   (float*)nullptr, (float*)nullptr);
            });
            if (rc) return rc;
        }
        if (y_bar) {
            rc = ln.run(ADMM_K_FINAL, [&] {
                hipLaunchKernelGGL(admm::branch_sum_kernel, dim3(1024), dim3(kThreads), 0, s, vout, y_bar, ppb * MN, nbr);
            });
            if (rc) return rc;
        }
        return ln.finish();
    }
    float4* dxK = rho_bar ? reinterpret_cast<float4*>(ws + L.sln) : nullptr;   // the forward's s state is dead
    float* vbuf = y_bar ? reinterpret_cast<float*>(ws + L.hln) : nullptr;     // ... and its H^T y copies
    double* part = reinterpret_cast<double*>(ws + L.part);
    if (dxK) {
        rc = ln.run(ADMM_K_PREP, [&] { return admm::plane::launch_dx_lane(x_out, dxK, planes, s, &br); });
        if (rc) return rc;
    }
    rc = ln.run(ADMM_K_ADJ, [&] {
        return admm::plane::launch_plane_adj(x_bar, ws + L.F, ws + L.traj, dxK, reinterpret_cast<float4*>(ws + L.sbar),
                                             reinterpret_cast<float2*>(ws + L.vsl), vbuf, part,
                                             prm, K, planes, s, &br, masks);
    });
    if (rc) return rc;
    double* rt = reinterpret_cast<double*>(ws + L.rt);
    for (int i = 0; i < nbr; ++i) {
        rc = ln.run(ADMM_K_FINAL, [&] {
            launch_reduce_cols(s, part + 2 * (size_t)i * ppb, rt + 2 * i, (int)ppb, 2, reinterpret_cast<double*>(ws + L.rtmp));
        });
        if (rc) return rc;
        rc = ln.run(ADMM_K_FINAL, [&] {
            hipLaunchKernelGGL(admm::grads_final_kernel, dim3(1), dim3(64), 0, s, rt + 2 * i, (const double*)nullptr,
                               (const double*)nullptr, 0, prm + 4 * i, lambda_bar ? lambda_bar + i : nullptr,
                               rho_bar ? rho_bar + i : nullptr, (float*)nullptr);
        });
        if (rc) return rc;
    }
    if (y_bar) {
        rc = ln.run(ADMM_K_FINAL, [&] {
            hipLaunchKernelGGL(admm::branch_sum_kernel, dim3(1024), dim3(kThreads), 0, s, vbuf, y_bar, ppb * MN, nbr);
        });
        if (rc) return rc;
    }
    return ln.finish();
}

}  // namespace admm_capi
