// admm_capi.hip -- extern "C" boundary (include/admm_deconv.h) for the ADMM TV-deconvolution
// solve on MI355X.  Replaces tvd_fft / tvd_fft_gpu (/root/reference/src/ops/ops.jl:99-188).
//
// Host side: validates the call, carves the caller's workspace, and enqueues
//   SETUP  (twiddles + C, ops.jl:22-37)
//   PREP   (H^T y once + first line rFFT, ops.jl:71-81 / :168 first iteration)
//   K x COLUMN, (K-1) x LINE, 1 x FINAL                (ops.jl:166-174)
// on the caller's stream.  Nothing is allocated and nothing synchronises unless the optional
// profiler is on.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <mutex>
#include <unordered_map>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/admm_deconv.h"
#include "admm_kernels.hip"
#include "admm_generic.hip"
#include "admm_backward.hip"
#include "admm_generic_bwd.hip"
#include "plane_api.hpp"
#include "smooth_api.hpp"
#include "resident_api.hpp"
#include "layout.hpp"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
}  // namespace

namespace admm_internal {
// error reporting for the other translation units of the library (metrics_capi.hip)
int fail_msg(int code, const char* msg) {
    g_err = msg;
    return code;
}
}  // namespace admm_internal

namespace {
int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

using namespace admm::layout;
constexpr int kGenMax = 4096;

// Library options (admm_set_option; process-global, read at each call).  The defaults are the tuned
// choices; the others exist for tests (fused vs 2-pass) and tuning experiments.  A recording stores
// the option values it was made with, and its replay rejects a change (RecTag below).
std::atomic<int> g_opt[ADMM_OPT_COUNT] = {{1}, {1}, {0}, {0}, {0}, {0}, {0}, {1}, {1}, {-1}};
int opt(int k) { return g_opt[k].load(std::memory_order_relaxed); }

// ADMM_OPT_FUSED = 0 forces the 2-pass path (tests compare the two).
bool fused_enabled() { return opt(ADMM_OPT_FUSED) != 0; }
// ADMM_OPT_FUSED_ADJ = 0 keeps the 2-pass reverse sweep (line_adj + column) on a fused trajectory
bool fused_adj_enabled() { return opt(ADMM_OPT_FUSED_ADJ) != 0; }

// ---- tile-size policy ------------------------------------------------------------------------
// T = lines per line-kernel block (power of two dividing N); KB = slots per column-kernel block.
int line_T(int M, int N) {
    int pref = M <= 512 ? 8 : 4;
    const int v = opt(ADMM_OPT_LINE_T);
    if (v == 2 || v == 4 || v == 8 || v == 16) pref = v < pref ? v : pref;
    return N < pref ? N : pref;
}
size_t line_lds(int M, int T) {
    const size_t L = M / 2;
    return (size_t)M * 8 + 3 * (size_t)(T + 2) * L * 8;
}
size_t fwdinv_lds(int M, int T) { return (size_t)M * 8 + 2 * (size_t)T * (M / 2) * 8; }
int max_q(int NN) {
    switch (NN) {
#define X(v) case v: return admm::plan_max_q<v, false>();
        X(2) X(4) X(8) X(16) X(32) X(64) X(128) X(256) X(512) X(1024)
#undef X
    }
    return NN;
}
// column block size: 1024 threads for long columns, so that a block covers >= 64 B of every row
// (256 threads at N = 512 gave 4 slots = 32 B per row); ADMM_OPT_COL_THREADS overrides (256 or 1024)
int column_threads(int N) {
    int nt = N >= 512 ? 1024 : 256;
    const int v = opt(ADMM_OPT_COL_THREADS);
    if (v == 256 || (v == 1024 && N >= 256)) nt = v;
    return nt;
}
int column_KB(int M, int N) {
    int KB = column_threads(N) / max_q(N);
    if (KB > M / 2) KB = M / 2;
    if (KB > 32) KB = 32;
    return KB;
}
// reverse sweep line tile: the isotropic adjoint kernels (ISO_ADJ_A / _B) run best with 4 lines per
// block (c5 iso: 55.4 -> 51.9 ms of adjoint per step, tools/iso_knobs.sh); the rest keeps line_T
int bwd_line_T(int M, int N, bool iso) {
    const int t = line_T(M, N);
    return iso && t > 4 ? 4 : t;
}
size_t column_lds(int N, int KB) { return (size_t)N * 16 + (size_t)KB * (N + 1) * 8; }
size_t iso_a_lds(int M, int T) { return (size_t)M * 8 + 3 * (size_t)(T + 1) * (M / 2) * 8; }
size_t iso_b_lds(int M, int T) { return (size_t)M * 8 + (size_t)(2 * T + 1) * M * 4 + 2 * (size_t)T * (M / 2) * 8; }

// ---- profiler -------------------------------------------------------------------------------
struct Prof {
    bool on = false;
    double ms[ADMM_K_COUNT] = {};
    long long n[ADMM_K_COUNT] = {};
    std::mutex mu;
} g_prof;

struct PendingEv {
    int cls;
    hipEvent_t a, b;
};

struct Launcher {
    hipStream_t s;
    bool prof;
    std::vector<PendingEv> ev;
    // `launch` may return void or an int status: the template dispatchers (launch_line, launch_column,
    // ...) return non-zero when no instance matches the requested tile, in which case nothing was
    // enqueued and the call must fail instead of returning unwritten outputs.
    template <typename F>
    int run(int cls, F&& launch) {
        PendingEv p{cls, nullptr, nullptr};
        if (prof) {
            hipEventCreate(&p.a);
            hipEventCreate(&p.b);
            hipEventRecord(p.a, s);
        }
        int lrc = 0;
        hipError_t e = hipSuccess;
        using R = decltype(launch());
        if constexpr (std::is_void_v<R>) {
            launch();
        } else if constexpr (std::is_same_v<R, hipError_t>) {
            e = launch();   // the plane launchers report hipGetLastError() themselves
        } else {
            lrc = (int)launch();
        }
        if (e == hipSuccess) e = hipGetLastError();
        if (prof) {
            hipEventRecord(p.b, s);
            ev.push_back(p);
        }
        if (e != hipSuccess) return fail(ADMM_E_HIP, "kernel launch (class %d) failed: %s", cls, hipGetErrorString(e));
        if (lrc != 0) return fail(ADMM_E_UNSUPPORTED, "no kernel instance for this tile (class %d, status %d)", cls, lrc);
        return ADMM_OK;
    }
    int finish() {
        if (!prof) return ADMM_OK;
        hipError_t e = hipStreamSynchronize(s);
        std::lock_guard<std::mutex> lk(g_prof.mu);
        for (auto& p : ev) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
                g_prof.ms[p.cls] += ms;
                g_prof.n[p.cls] += 1;
            }
            hipEventDestroy(p.a);
            hipEventDestroy(p.b);
        }
        ev.clear();
        if (e != hipSuccess) return fail(ADMM_E_HIP, "stream sync failed: %s", hipGetErrorString(e));
        return ADMM_OK;
    }
};

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

int launch_line_fwd(int L, int T, dim3 g, size_t lds, hipStream_t s, const float* src, float2* spec,
                    const float2* twM, int N) {
#define X(l, t)                                                            \
    if (L == l && T == t) {                                                \
        set_lds(line_fwd_kernel<l, t>, lds);                               \
        line_fwd_kernel<l, t><<<g, kThreads, lds, s>>>(src, spec, twM, N); \
        return 0;                                                          \
    }
    ADMM_LT_CASES(X)
#undef X
    return -1;
}

int launch_line_inv(int L, int T, dim3 g, size_t lds, hipStream_t s, const float2* spec, float* dst,
                    const float2* twM, int N) {
#define X(l, t)                                                            \
    if (L == l && T == t) {                                                \
        set_lds(line_inv_kernel<l, t>, lds);                               \
        line_inv_kernel<l, t><<<g, kThreads, lds, s>>>(spec, dst, twM, N); \
        return 0;                                                          \
    }
    ADMM_LT_CASES(X)
#undef X
    return -1;
}

int launch_line(int L, int T, dim3 g, size_t lds, hipStream_t s, const float2* spec1, float2* spec0,
                const float* so, float* sn, const float* hty, const float2* twM, int N, const float* prm,
                int sz) {
#define X(l, t)                                                                                          \
    if (L == l && T == t) {                                                                              \
        set_lds(line_kernel<l, t>, lds);                                                                 \
        line_kernel<l, t><<<g, kThreads, lds, s>>>(spec1, spec0, so, sn, hty, twM, N, prm, sz);    \
        return 0;                                                                                        \
    }
    ADMM_LT_CASES(X)
#undef X
    return -1;
}

int launch_iso_a(int L, int T, dim3 g, size_t lds, hipStream_t s, const float2* spec1, const float* so, float* sn,
                 const float* fmap, float* part, const float2* twM, int N, int planes, int G, int sz) {
#define X(l, t)                                                                                             \
    if (L == l && T == t) {                                                                                 \
        set_lds(iso_a_kernel<l, t>, lds);                                                                   \
        iso_a_kernel<l, t><<<g, kThreads, lds, s>>>(spec1, so, sn, fmap, part, twM, N, planes, G, sz);     \
        return 0;                                                                                           \
    }
    ADMM_LT_CASES(X)
#undef X
    return -1;
}

int launch_iso_b(int L, int T, dim3 g, size_t lds, hipStream_t s, const float* sn, const float* fmap,
                 const float* hty, float2* spec0, const float2* twM, int N, const float* prm) {
#define X(l, t)                                                                               \
    if (L == l && T == t) {                                                                   \
        set_lds(iso_b_kernel<l, t>, lds);                                                     \
        iso_b_kernel<l, t><<<g, kThreads, lds, s>>>(sn, fmap, hty, spec0, twM, N, prm);      \
        return 0;                                                                             \
    }
    ADMM_LT_CASES(X)
#undef X
    return -1;
}

template <int MUL, bool SAVE, bool ACCQ>
int launch_column_t(int N, dim3 g, size_t lds, hipStream_t s, const float2* src, float2* dst, const float* C,
                    const float2* G, const float2* twN, int L, int KB, float cs, float2* vsave, double* Qp) {
    const int nt = column_threads(N);
#define X(v)                                                                                                   \
    if (N == v && nt == kThreads) {                                                                            \
        set_lds(column_kernel<v, MUL, SAVE, ACCQ>, lds);                                                       \
        column_kernel<v, MUL, SAVE, ACCQ><<<g, kThreads, lds, s>>>(src, dst, C, G, twN, L, KB, cs, vsave, Qp); \
        return 0;                                                                                              \
    }
    ADMM_N_CASES(X)
#undef X
#define X(v)                                                                                                   \
    if (N == v && nt == 1024) {                                                                                \
        set_lds(column_kernel<v, MUL, SAVE, ACCQ, 1024>, lds);                                                 \
        column_kernel<v, MUL, SAVE, ACCQ, 1024><<<g, 1024, lds, s>>>(src, dst, C, G, twN, L, KB, cs, vsave, Qp); \
        return 0;                                                                                              \
    }
    X(256) X(512) X(1024)
#undef X
    return -1;
}

// mode: 0 = x-update C, 1 = conj(Sigma_c) (H^T), 2 = Sigma_c (H), 3 = C + save spectrum, 4 = C + accumulate Q
int launch_column(int N, int mode, dim3 g, size_t lds, hipStream_t s, const float2* src, float2* dst,
                  const float* C, const float2* G, const float2* twN, int L, int KB, float cs,
                  float2* vsave = nullptr, double* Qp = nullptr) {
    switch (mode) {
        case 0: return launch_column_t<0, false, false>(N, g, lds, s, src, dst, C, G, twN, L, KB, cs, vsave, Qp);
        case 1: return launch_column_t<1, false, false>(N, g, lds, s, src, dst, C, G, twN, L, KB, cs, vsave, Qp);
        case 2: return launch_column_t<2, false, false>(N, g, lds, s, src, dst, C, G, twN, L, KB, cs, vsave, Qp);
        case 3: return launch_column_t<0, true, false>(N, g, lds, s, src, dst, C, G, twN, L, KB, cs, vsave, Qp);
        case 4: return launch_column_t<0, false, true>(N, g, lds, s, src, dst, C, G, twN, L, KB, cs, vsave, Qp);
    }
    return -1;
}

int check_shape(int M, int N, int P, int B, int kh, int kw, int iso) {
    if (P < 1 || B < 1 || M < 1 || N < 1) return fail(ADMM_E_INVALID, "sizes must be positive (M=%d N=%d P=%d B=%d)", M, N, P, B);
    if (kh < 0 || kw < 0 || ((kh == 0) != (kw == 0)))
        return fail(ADMM_E_INVALID, "PSF size must be both zero (empty PSF) or both positive (kh=%d kw=%d)", kh, kw);
    // M, N >= 2 as in the reference (ops.jl:32-33 index the second row / column of the D stencils)
    if (M < 2 || N < 2 || M > kGenMax || N > kGenMax)
        return fail(ADMM_E_UNSUPPORTED, "this build supports 2<=M<=%d, 2<=N<=%d (got M=%d N=%d)", kGenMax, kGenMax, M, N);
    if (kh > M || kw > N)
        return fail(ADMM_E_UNSUPPORTED, "PSF %dx%d larger than the image (kh<=M, kw<=N required, as pad_constant in ops.jl:25)", kh, kw);
    if (iso && (size_t)P * B > 65535)
        return fail(ADMM_E_UNSUPPORTED, "isotropic prox couples the batch: at most 65535 planes per call");
    return ADMM_OK;
}

// Planes per launch sequence.  The 2-pass kernels index planes by blockIdx.y (<= 65535), so a larger
// anisotropic forward runs as consecutive chunks of this many planes through one chunk-sized workspace
// (planes are independent, ops.jl:168-173).  A multiple of 256: every chunk but the last fills whole
// waves of the fused kernel (one workgroup per CU).
constexpr size_t kChunkPlanes = 255 * 256;
size_t launch_planes(size_t planes) { return planes < kChunkPlanes ? planes : kChunkPlanes; }
// The isotropic prox couples the whole batch through the per-pixel norm (ops.jl:6), so an isotropic
// batch is never split: it runs as one launch sequence of up to 65535 planes (check_shape's limit).
size_t chunk_planes(size_t planes, bool iso) { return iso ? planes : launch_planes(planes); }

}  // namespace

extern "C" {

int admm_abi_version(void) { return ADMM_ABI_VERSION; }

const char* admm_last_error(void) { return g_err.c_str(); }

int admm_tvd_workspace_bytes(int M, int N, int P, int B, int kh, int kw, int iso, size_t* out_bytes) {
    if (!out_bytes) return fail(ADMM_E_INVALID, "out_bytes is NULL");
    int rc = check_shape(M, N, P, B, kh, kw, iso);
    if (rc) return rc;
    *out_bytes = make_layout(M, N, chunk_planes((size_t)P * B, iso != 0), kh > 0, iso != 0).total;
    return ADMM_OK;
}

}  // extern "C"

namespace {

// Trajectory recorded by the forward for the backward (all optional).
struct Traj {
    float* s = nullptr;      // (K-1) x planes x 2 x M x N : s_k for k = 1..K-1
    float2* v = nullptr;     // K x planes x N x M/2        : forward dim-2 spectra (h_bar only)
    double2* sig = nullptr;  // (M/2+1) x N                 : top-left PSF spectrum (h_bar only)
    float* nrm = nullptr;    // (K-1) x M x N               : isotropic batch norm of s_k (iso only)
    unsigned* m = nullptr;   // (K-1) x planes x 16 x 512   : ST mask bytes of s_k instead of s (fused only)
    bool iso_lane = false;   // isotropic 256 x 256: s and nrm lane-native (plane_iso.hip), for the fused adjoint
};

// ---- path selection: ONE decision table for every entry point -----------------------------------------------
// Which kernels a call runs is decided here and nowhere else; run_forward / run_forward_generic / run_backward
// only execute the plan, and admm_query_paths (include/admm_deconv.h) returns it to tests without a GPU.
// Inputs: shape, prox, PSF, what the call is (plain forward, recording with ADMM_REC_* flags, combined
// backward with or without h_bar / rho_bar) and the library options.
struct PathIn {
    int M, N;
    bool iso, psf;
    int mode;            // ADMM_MODE_FORWARD, ADMM_MODE_RECORD, ADMM_MODE_BACKWARD
    int rec_flags;       // ADMM_REC_* (record)
    bool h_bar, rho_bar; // backward: gradients asked for
    size_t planes;       // P * B of the call (0: unknown, no plane-count rule)
};
// Plane counts from which the one-workgroup-per-plane paths beat the 2-pass kernels (ADMM_OPT_MIN_PLANES = -1).
// A per-plane grid uses one CU per plane for the whole solve, so below about one CU wave it leaves CUs idle
// while the 2-pass kernels spread every plane over many workgroups.  Measured on MI355X (tools/time_small.py,
// profiles/r04_small_batch_paths.jsonl; K = 25 forward, K = 50 recording + sweep):
//   fused 256^2 anisotropic  forward 96 planes 1.32 vs 1.34 ms, 64: 1.29 vs 1.07; recording + sweep 96: 5.55 vs
//                            6.24, 64: 5.34 vs 4.75  -> 96
//   fused_iso 256^2          128: 2.03 vs 2.13, 64: 1.84 vs 1.40  -> 112
//   resident 250^2           192: 2.53 vs 2.96, 128: 2.48 vs 1.99; 128^2 256: 0.88 vs 0.93, 128: 0.84 vs 0.62
//                            -> 192 for sides >= 128 (smaller sides: every batch, the per-plane latency is small)
//                            (sides < 128: 96^2 0.43 vs 0.40 at 1..16 planes, 64^2 and 32^2 faster at every count)
//   resident_iso             256 planes: 250^2 3.94 vs 5.78, 120^2 1.04 vs 1.53, 64^2 x 512 0.80 vs 0.96;
//                            250^2 x 64 4.41 vs 1.84 (before its A / B row walkers)  -> 256
enum MinPlanesFor { kMinFused, kMinFusedIso, kMinResident, kMinResidentIso };
bool enough_planes(const PathIn& q, MinPlanesFor which) {
    const int o = opt(ADMM_OPT_MIN_PLANES);
    if (q.planes == 0 || o == 0) return true;
    if (o > 0) return q.planes >= (size_t)o;
    switch (which) {
        case kMinFused: return q.planes >= 96;
        case kMinFusedIso: return q.planes >= 112;
        case kMinResident: return std::max(q.M, q.N) < 128 || q.planes >= 192;
        case kMinResidentIso: return q.planes >= 256;
    }
    return true;
}
struct PathPlan {
    bool want_h = false;     // the forward records the dim-2 spectra h_bar needs (2-pass column pass)
    bool ln_traj = false;    // the fused 256^2 forward records s lane-native
    bool masks = false;      // ADMM_REC_MASKS honoured: ST mask bits (aniso) / lane-native s and |s| (iso)
    bool iso_lane = false;   // the fused isotropic trajectory + sweep
    int fwd = 0;             // ADMM_PATH_* of the forward
    int bwd = 0;             // ADMM_PATH_SWEEP_* of the reverse sweep (0: none)
};
// the trajectory a recording keeps, as run_forward sees it (pointers only matter as null / non-null)
struct TrajFlags {
    bool s, v, nrm, m, iso_lane;
};
TrajFlags traj_flags(const PathIn& q, const PathPlan& pl) {
    if (q.mode == ADMM_MODE_FORWARD) return {false, false, false, false, false};
    return {true, pl.want_h, q.iso, pl.masks && !q.iso, pl.iso_lane};
}
// forward rules, first match wins
struct FwdRule {
    int path;
    bool (*applies)(const PathIn&, const TrajFlags&);
};
const FwdRule kFwdRules[] = {
    // runtime-length shapes: the CU-resident solve (admm_resident.hip) where compiled and measured faster,
    // anisotropic and recording neither dim-2 spectra, norms nor mask bits (it writes s_k into the slots)
    // (and the small power-of-two squares it compiled: 32, 64, 128; it needs no spectra buffers, so it runs on
    // either layout)
    {ADMM_PATH_RESIDENT, [](const PathIn& q, const TrajFlags& t) {
         return !q.iso && !t.v && !t.nrm && !t.m && opt(ADMM_OPT_RESIDENT) != 0 &&
                (!generic_shape(q.M, q.N) || opt(ADMM_OPT_SMOOTH) != 0) &&
                admm::rs::has_shape(q.M, q.N, opt(ADMM_OPT_RESIDENT) >= 2) && enough_planes(q, kMinResident);
     }},
    // isotropic: the split-iteration CU-resident solve (resident_iso_kernel, one launch per iteration with the
    // norm kernel between); it records s_k and |s_k| in the natural layout the 2-pass / runtime sweeps read
    {ADMM_PATH_RESIDENT_ISO, [](const PathIn& q, const TrajFlags& t) {
         return q.iso && !t.v && opt(ADMM_OPT_RESIDENT) != 0 && (!generic_shape(q.M, q.N) || opt(ADMM_OPT_SMOOTH) != 0) &&
                admm::rs::has_iso_shape(q.M, q.N, opt(ADMM_OPT_RESIDENT) >= 2) && enough_planes(q, kMinResidentIso);
     }},
    // compile-time-plan kernels when this build has either length (admm_smooth.hip), else runtime plans
    {ADMM_PATH_SMOOTH, [](const PathIn& q, const TrajFlags&) {
         return generic_shape(q.M, q.N) && opt(ADMM_OPT_SMOOTH) != 0 &&
                (admm::sm::has_length(q.M) || admm::sm::has_length(q.N));
     }},
    {ADMM_PATH_RUNTIME, [](const PathIn& q, const TrajFlags&) { return generic_shape(q.M, q.N); }},
    // 256 x 256 anisotropic: one workgroup per plane runs all K iterations (plane_kernel.hip)
    {ADMM_PATH_FUSED, [](const PathIn& q, const TrajFlags& t) {
         return fused_shape(q.M, q.N, q.iso) && !t.v && fused_enabled() && enough_planes(q, kMinFused);
     }},
    // 256 x 256 isotropic: split-iteration per-plane kernels (plane_iso.hip); a recording only in its own
    // lane-native layout (the fused sweep's)
    {ADMM_PATH_FUSED_ISO, [](const PathIn& q, const TrajFlags& t) {
         return q.iso && fused_tables_shape(q.M, q.N) && (!t.s || t.iso_lane) && !t.v && fused_enabled() &&
                enough_planes(q, kMinFusedIso);
     }},
    {ADMM_PATH_2PASS_ISO, [](const PathIn& q, const TrajFlags&) { return q.iso; }},
    {ADMM_PATH_2PASS, [](const PathIn&, const TrajFlags&) { return true; }},
};

PathPlan plan_paths(const PathIn& q) {
    PathPlan pl;
    const bool rec = q.mode != ADMM_MODE_FORWARD;
    if (rec) {
        pl.want_h = (q.mode == ADMM_MODE_RECORD ? (q.rec_flags & ADMM_REC_HBAR) != 0 : q.h_bar) && q.psf;
        // the fused kernel records s in its lane-native layout (no dim-2 spectra: not with h_bar)
        pl.ln_traj = fused_shape(q.M, q.N, q.iso) && fused_enabled() && !pl.want_h && enough_planes(q, kMinFused);
        // mask-bit trajectory (fused forward + fused reverse sweep): asked for by a recording (ADMM_REC_MASKS),
        // taken by the combined call whenever rho_bar is not wanted; isotropic at 256 x 256 the same flag
        // selects the split-iteration trajectory (s and |s| lane-native) for the fused isotropic sweep
        const bool iso_ok = q.iso && fused_tables_shape(q.M, q.N) && !pl.want_h && fused_enabled() && fused_adj_enabled() &&
                            enough_planes(q, kMinFusedIso);
        const bool masks_ok = (pl.ln_traj && !q.iso && fused_adj_enabled()) || iso_ok;
        pl.masks = masks_ok && (q.mode == ADMM_MODE_RECORD ? (q.rec_flags & ADMM_REC_MASKS) != 0 : !q.rho_bar);
        pl.iso_lane = pl.masks && q.iso;
    }
    const TrajFlags t = traj_flags(q, pl);
    for (const FwdRule& r : kFwdRules)
        if (r.applies(q, t)) {
            pl.fwd = r.path;
            break;
        }
    if (rec) {
        if (pl.ln_traj && !q.iso && fused_adj_enabled()) pl.bwd = ADMM_PATH_SWEEP_FUSED;         // plane256_adj_kernel
        else if (pl.iso_lane) pl.bwd = ADMM_PATH_SWEEP_FUSED_ISO;                                   // plane256_isoadj
        else if (generic_shape(q.M, q.N)) pl.bwd = q.iso ? ADMM_PATH_SWEEP_RUNTIME_ISO : ADMM_PATH_SWEEP_RUNTIME;
        else pl.bwd = q.iso ? ADMM_PATH_SWEEP_2PASS_ISO : ADMM_PATH_SWEEP_2PASS;
    }
    return pl;
}

// Shared forward: everything admm_tvd_forward_f32 does, plus optional trajectory recording.
// Returns the Launcher's status; `ln` keeps the events for the profiler.
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
// lines per block: the largest of 8, 4, 2, 1 dividing N with T * M <= 4096 (LDS ~ 24 T M bytes)
// options ADMM_OPT_GEN_TM (max T x M of a line block), ADMM_OPT_GEN_KN (max KB x N of a column block)
int gen_opt(int k, int dflt) {
    const int v = opt(k);
    return v >= 256 && v <= 8192 ? v : dflt;
}
int gen_T(int M, int N) {
    // 2048: smaller blocks, more of them resident per CU (480x640: 1.3x over 4096, tools/gen_knobs.sh).
    // T need not divide N (ragged last block): 250 x 250 ran 2-line blocks when it had to.
    const int tm = gen_opt(ADMM_OPT_GEN_TM, 2048);
    for (int t = 8; t > 1; t >>= 1)
        if (t * M <= tm && t <= N) return t;
    return 1;
}
// line blocks per plane: the last block of a plane may hold fewer than T lines (N need not divide by T)
int gen_nb(int N, int T) { return (N + T - 1) / T; }
int gen_KB(int M, int N) {
    // 1024 points per column block: with the XCD-aware block order, smaller blocks won at every size
    // measured (480x640 column pass 3.29 -> 2.92 ms; 256 / 512 / 2048+ slower, tools/time_generic.py)
    int kb = gen_opt(ADMM_OPT_GEN_KN, 1024) / N;
    kb = kb < 1 ? 1 : (kb > 16 ? 16 : kb);
    return kb > M / 2 + 1 ? M / 2 + 1 : kb;
}
// dynamic LDS of the runtime-length kernels: ping-pong FFT buffers (+ the two D^T channels of the
// update kernels) + the twiddle table staged by gen::stage_tw (8 n bytes, 8-B aligned)
size_t gen_lds_line(int M, int T, bool upd) {
    // A, B hold ceil(T / 2) paired complex transforms (gen::pack_real: two real lines per transform)
    const size_t base = (size_t)2 * ((T + 1) / 2) * M * 8 + (upd ? (size_t)(2 * T + 1) * M * 4 : 0);
    return ((base + 7) & ~size_t(7)) + (size_t)M * 8;
}
size_t gen_lds_col(int N, int KB) { return (size_t)2 * KB * N * 8 + (size_t)N * 8; }

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
                const Traj& tr, const admm_batch_reducer* red, int fwd_path) {
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

    rc = ln.run(ADMM_K_SETUP, [&] {
        const size_t lds = (size_t)(M + N) * 16 + (kh * kw <= admm::kSetupPsfLds ? (size_t)kh * kw * 4 : 0);
        const int nb = (int)(((size_t)(L + 1) * N + kThreads - 1) / kThreads);
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
        void* tables = ws + lay.F;
        rc = ln.run(ADMM_K_SETUP, [&] { return pk::launch_tables(Ct, Gt, tables, s); });
        if (rc) return rc;
        rc = ln.run(ADMM_K_PLANE, [&] {
            return pk::launch_plane(y, x_out, tables, kh > 0, spec0, reinterpret_cast<float4*>(sbuf[0]), prm, maxit,
                                   planes, s, tr.m ? nullptr : reinterpret_cast<float4*>(tr.s),
                                   opt(ADMM_OPT_PLANE_STAGGER), nullptr, tr.m);
        });
        return rc;
    }
    if (path == ADMM_PATH_FUSED_ISO) {
        // isotropic at 256 x 256: the split-iteration per-plane kernels (plane_iso.hip), the spectrum
        // resident in the CU; per iteration one plane256_iso_kernel and one iso_norm_kernel (batch norm)
        namespace pk = admm::plane;
        void* tables = ws + lay.F;
        rc = ln.run(ADMM_K_SETUP, [&] { return pk::launch_tables(Ct, Gt, tables, s); });
        if (rc) return rc;
        float2* fl = reinterpret_cast<float2*>(ws + lay.fmap);
        float2* ql = reinterpret_cast<float2*>(spec1);
        // recording: s_{k+1} into trajectory slot k, |s_{k+1}| into norm slot k (lane-native)
        float4* st = reinterpret_cast<float4*>(tr.iso_lane ? tr.s : sbuf[0]);
        const size_t tslot = tr.iso_lane ? planes * MN / 2 : 0;   // float4 per slot
        for (int k = 0; k < maxit; ++k) {
            rc = ln.run(ADMM_K_PLANE, [&] {
                return pk::launch_plane_iso(y, x_out, tables, kh > 0, spec0, st + (k > 0 ? (size_t)(k - 1) * tslot : 0),
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
    const int Tu = (M == 512 && T > 4) ? 4 : T;
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
                                    maxit, opt(ADMM_OPT_PLANE_STAGGER));
        });
    }
    // PREP: spectrum of y; with a PSF, H^T y = F^-1 conj(Sigma_c) F y (line, column, line)
    rc = ln.run(ADMM_K_PREP, [&] { return launch_line_fwd(L, T, gl, flds, s, y, spec0, twM, N); });
    if (rc) return rc;
    const float2* first = spec0;
    float cs1 = 1.0f;
    if (kh > 0) {
        rc = ln.run(ADMM_K_PREP, [&] { return launch_column(N, 1, gc, clds, s, spec0, spec1, Ct, Gt, twN, L, KB, 1.0f); });
        if (rc) return rc;
        rc = ln.run(ADMM_K_PREP, [&] { return launch_line_inv(L, T, gl, flds, s, spec1, hty, twM, N); });
        if (rc) return rc;
        first = spec1;          // = F_dim1(H^T y) / M
        cs1 = (float)M;
    }
    const size_t sstride = np * 2 * MN;   // one trajectory slot of s
    for (int it = 1; it <= maxit; ++it) {
        float2* vsave = tr.v ? tr.v + (size_t)(it - 1) * np * N * L : nullptr;
        rc = ln.run(ADMM_K_COLUMN, [&] {
            return launch_column(N, vsave ? 3 : 0, gc, clds, s, it == 1 ? first : spec0, spec1, Ct, Gt, twN, L, KB,
                          it == 1 ? cs1 : 1.0f, vsave);
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
                return launch_line(L, Tu, dim3(N / Tu, (unsigned)np), llds, s, spec1, spec0, so, sn, hty, twM, N, prm,
                            it == 1 ? 1 : 0);
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
                return launch_iso_b(L, T, gl, iso_b_lds(M, T), s, sn, fmap, hty, spec0, twM, N, prm);
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
    // PREP: spectrum of H^T y (with a PSF: F^-1 conj(Sigma_c) F y first, ops.jl:71-81)
    if (!res || kh > 0) {
        rc = line_fwd(y, spec0);
        if (rc) return rc;
    }
    if (kh > 0) {
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
        if (!res) {
            rc = line_fwd(hty, spec0);
            if (rc) return rc;
        }
    }
    const int ng = iso_ngroups(planes);
    const size_t sstride = planes * 2 * MN;   // one trajectory slot of s
    if (path == ADMM_PATH_RESIDENT_ISO)
        return run_resident_iso(ln, M, N, planes, hty, sbuf[0], reinterpret_cast<float*>(spec1), fmap, x_out, Ct, twM, twN,
                                prm, maxit, tr, red);
    if (res) {
        return ln.run(ADMM_K_PLANE, [&] {
            return admm::rs::launch(M, N, planes, s, hty, sbuf[0], sbuf[1], tr.s, sstride, x_out, Ct, twM, twN, prm, maxit,
                                    opt(ADMM_OPT_PLANE_STAGGER));
        });
    }
    for (int it = 1; it <= maxit; ++it) {
        // trajectory for h_bar: the dim-2 spectrum of iteration it before the multiply
        float2* vsave = tr.v ? tr.v + (size_t)(it - 1) * planes * N * H : nullptr;
        rc = ln.run(ADMM_K_COLUMN, [&] {
            if (smc && !vsave) return admm::sm::launch_column(M, N, planes, s, spec0, spec1, Ct, Gt, twN, 1.0f, 0, opt(ADMM_OPT_SMOOTH));
            hipLaunchKernelGGL(g::column_kernel, gc, dim3(256), lcol, s, spec0, spec1, Ct, Gt, twN, pN, H, KB,
                               vsave ? 4 : 0, 1.0f, vsave, (double*)nullptr);
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
                if (sml) return admm::sm::launch_line_upd(M, N, planes, s, xg, so, sn, hty, spec0, twM, prm, it == 1 ? 1 : 0);
                hipLaunchKernelGGL(g::line_upd_kernel, gl, dim3(256), lup, s, xg, so, sn, hty, spec0, twM, pM, N, T, prm,
                                   it == 1 ? 1 : 0);
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
            hipLaunchKernelGGL(g::iso_b_kernel, gl, dim3(256), lup, s, sa, fmap, hty, spec0, twM, pM, N, T, prm);
        });
        if (rc) return rc;
    }
    return ADMM_OK;
}

int check_common(const float* y, float* x, int maxit) {
    if (!y || !x) return fail(ADMM_E_INVALID, "y and x_out must be device pointers");
    if (maxit < 0) return fail(ADMM_E_INVALID, "maxit must be >= 0 (got %d)", maxit);
    if ((reinterpret_cast<uintptr_t>(y) & 15) || (reinterpret_cast<uintptr_t>(x) & 15))
        return fail(ADMM_E_INVALID, "y and x_out must be 16-byte aligned");
    return ADMM_OK;
}

int check_ws(void* workspace, size_t have, size_t need) {
    if (!workspace || have < need) return fail(ADMM_E_WORKSPACE, "workspace too small: need %zu bytes, got %zu", need, have);
    if ((reinterpret_cast<uintptr_t>(workspace) & 255) != 0) return fail(ADMM_E_WORKSPACE, "workspace must be 256-byte aligned");
    return ADMM_OK;
}

// backward workspace = forward layout + trajectory + reverse-sweep buffers
struct BwdLayout {
    Layout f;
    size_t traj_s, traj_v, sig, sbA, sbB, vsum, rpart, Qp, Q, hpart, hcorr, hA, rt, total;
    size_t traj_n, wbar, Rmap, Rpart;   // isotropic only
    size_t rtmp;                        // two-stage column sums (kRedParts x columns doubles)
    int nblk_line, nblk_corr, TY;
    int nblk_isoA, nblk_isoR;           // isotropic: per-step partial rows = nblk_isoA + nblk_isoR
};

constexpr int kIsoAdjRBlocks = 256;     // ISO_ADJ_R grid (tau_bar partial rows per step)
constexpr int kRedParts = 256;          // first-stage blocks per column of a long column sum

BwdLayout make_bwd_layout(int M, int N, size_t planes, int kh, int kw, int maxit, bool want_h, bool iso,
                          bool masks = false) {
    BwdLayout b{};
    const BwdHead hd = bwd_head(M, N, planes, kh, maxit, want_h, iso, masks);
    b.f = hd.f;
    b.traj_s = hd.traj_s, b.traj_v = hd.traj_v, b.sig = hd.sig, b.sbA = hd.sbA, b.sbB = hd.sbB, b.vsum = hd.vsum;
    b.traj_n = hd.traj_n;
    size_t off = hd.end;
    auto take = [&](size_t bytes) {
        size_t o = off;
        off = align_up(off + bytes);
        return o;
    };
    const size_t MN = (size_t)M * N;
    const int K = maxit < 1 ? 1 : maxit;
    const bool gen = generic_shape(M, N);
    const int T = gen ? gen_T(M, N) : bwd_line_T(M, N, iso);
    const bool hq = want_h && kh > 0;
    if (iso) {
        const size_t ng = iso_ngroups(planes);
        b.wbar = take(planes * MN * 4);   // vbar_k handed from ISO_ADJ_A to ISO_ADJ_B
        b.Rmap = take(MN * 4);
        b.Rpart = take(ng * MN * 4);
        b.nblk_isoA = (int)(ng * gen_nb(N, T));
        b.nblk_isoR = kIsoAdjRBlocks;
        b.nblk_line = b.nblk_isoA + b.nblk_isoR;
        if (b.nblk_line < 512) b.nblk_line = 512;   // the fused sweep's 512 tau_bar rows per step (plane_iso.hip)
    } else {
        b.nblk_line = (int)(planes * gen_nb(N, T));
    }
    b.rpart = take((size_t)K * b.nblk_line * 2 * 8);
    b.Qp = hq ? take(planes * (size_t)(M / 2 + 1) * N * 8) : 0;   // fp64 accumulators
    b.Q = hq ? take((size_t)(M / 2 + 1) * N * 8) : 0;
    b.TY = 1;   // h_bar correlation tile: the largest of 8, 4, 2, 1 lines dividing N
    for (int t = 8; t > 1; t >>= 1)
        if (N % t == 0) {
            b.TY = t;
            break;
        }
    b.nblk_corr = (int)(planes * (N / b.TY));
    b.hpart = kh > 0 ? take((size_t)b.nblk_corr * kh * kw * 8) : 0;
    b.hcorr = kh > 0 ? take((size_t)kh * kw * 8) : 0;
    b.hA = hq ? take((size_t)kh * kw * 8) : 0;
    b.rt = take(2 * 8);
    b.rtmp = take((size_t)kRedParts * (kh * kw > 2 ? kh * kw : 2) * 8);
    b.total = off;
    return b;
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
                    double* part, const float2* twM, int N, const float* prm, int first_k, int last_k, bool ln) {
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
                                                        N, prm, first_k, last_k);                        \
        return 0;                                                                                              \
    }
    ADMM_LT_CASES(X)
#undef X
    return -1;
}

int launch_iso_adj_a(int L, int T, dim3 g, size_t lds, hipStream_t s, const float2* spec1, const float* sk1,
                     const float* sk, const float* xK, const float* nrm1, const float* sb_in, float* wbar, float* vsum,
                     float* rpartial, double* part, const float2* twM, int N, int planes, int G, const float* prm,
                     int first_k, int last_k) {
#define X(l, t)                                                                                                 \
    if (L == l && T == t) {                                                                                     \
        set_lds(iso_adj_a_kernel<l, t>, lds);                                                                   \
        iso_adj_a_kernel<l, t><<<g, kThreads, lds, s>>>(spec1, sk1, sk, xK, nrm1, nullptr, sb_in, wbar, vsum,  \
                                                         rpartial, part, twM, N, planes, G, prm, first_k,  \
                                                         last_k);                                               \
        return 0;                                                                                               \
    }
    ADMM_LT_CASES(X)
#undef X
    return -1;
}

int launch_iso_adj_b(int L, int T, dim3 g, size_t lds, hipStream_t s, const float* wbar, const float* sb_in,
                     const float* sk1, const float* nrm1, const float* Rmap, float* sb_out, float2* spec0,
                     const float2* twM, int N, const float* prm) {
#define X(l, t)                                                                                                 \
    if (L == l && T == t) {                                                                                     \
        set_lds(iso_adj_b_kernel<l, t>, lds);                                                                   \
        iso_adj_b_kernel<l, t><<<g, kThreads, lds, s>>>(wbar, sb_in, sk1, nrm1, Rmap, sb_out, spec0, twM, N,    \
                                                         prm);                                                  \
        return 0;                                                                                               \
    }
    ADMM_LT_CASES(X)
#undef X
    return -1;
}


// ---- recordings: the path a forward-with-trajectory took, checked by its replay ----------------
// A recording lives in the caller's workspace; its replay must run the reverse sweep that matches the
// trajectory's layout (lane-native for the fused kernel, natural for the 2-pass and runtime-length
// paths) and the tile choices the workspace layout was sized with.  The host keeps one tag per
// recorded workspace; a replay whose arguments or library options differ from the recording's, or
// whose workspace holds no recording, fails with ADMM_E_INVALID instead of reading a foreign layout.
struct RecTag {
    int M, N, P, B, kh, kw, iso, maxit, want_h;
    int opts[ADMM_OPT_COUNT];
    // host-value lambda / rho of the recording (0, 0 for device-resident scalars, which the host cannot
    // read without a synchronisation): a replay with other host values is refused
    float lam, rho;
    int dev_scalars;
    int masks;   // the trajectory holds ST mask bytes (ADMM_REC_MASKS): no rho_bar
    int nbr;     // branches of a multi-branch recording (1: a single solve)
    bool operator==(const RecTag& o) const { return std::memcmp(this, &o, sizeof(RecTag)) == 0; }
};
std::mutex g_rec_mu;
std::unordered_map<const void*, RecTag> g_rec;
float g_dummy_scalar = 0.f;   // stands for "device-resident scalars" when a tag is rebuilt without them

RecTag make_tag(int M, int N, int P, int B, int kh, int kw, int iso, int maxit, bool want_h, const admm::ScalarSrc& sc) {
    RecTag t;
    std::memset(&t, 0, sizeof(t));
    t.M = M, t.N = N, t.P = P, t.B = B, t.kh = kh, t.kw = kw, t.iso = iso != 0, t.maxit = maxit, t.want_h = want_h;
    t.nbr = 1;
    t.dev_scalars = sc.lam != nullptr;
    if (!t.dev_scalars) t.lam = sc.lam_v, t.rho = sc.rho_v;
    for (int i = 0; i < ADMM_OPT_COUNT; ++i) t.opts[i] = opt(i);
    return t;
}
void rec_forget(const void* ws) {
    std::lock_guard<std::mutex> lk(g_rec_mu);
    g_rec.erase(ws);
}

int check_lam_rho(float lambda, float rho) {
    if (!std::isfinite(lambda) || !std::isfinite(rho)) return fail(ADMM_E_INVALID, "lambda and rho must be finite");
    return ADMM_OK;
}

int forward_impl(const float* y, float* x_out, int M, int N, int P, int B, const float* h, int kh, int kw,
                 const admm::ScalarSrc& sc, int iso, int maxit, void* workspace, size_t workspace_bytes, void* stream,
                 const admm_batch_reducer* reducer) {
    const admm_batch_reducer* red = (iso && reducer && reducer->fn) ? reducer : nullptr;
    if (h == nullptr) kh = kw = 0;
    int rc = check_shape(M, N, P, B, kh, kw, iso);
    if (rc) return rc;
    rc = check_common(y, x_out, maxit);
    if (rc) return rc;
    const size_t planes = (size_t)P * B;
    const size_t chunk = chunk_planes(planes, iso != 0);   // an isotropic batch is one chunk
    const Layout lay = make_layout(M, N, chunk, kh > 0, iso != 0);
    rc = check_ws(workspace, workspace_bytes, lay.total);
    if (rc) return rc;
    rec_forget(workspace);   // whatever was recorded there is overwritten now
    Launcher ln{reinterpret_cast<hipStream_t>(stream), g_prof.on, {}};
    const size_t MN = (size_t)M * N;
    // a sharded isotropic solve plans without the plane-count rule: every shard must take the same path, since
    // the fused and 2-pass kernels hand the reducer their sum maps in different layouts (lane-native float2 vs
    // natural), and uneven shards can fall on either side of a threshold
    const PathPlan pl = plan_paths({M, N, iso != 0, kh > 0, ADMM_MODE_FORWARD, 0, false, false, red ? 0 : planes});
    for (size_t p0 = 0; p0 < planes && rc == 0; p0 += chunk)
        rc = run_forward(ln, y + p0 * MN, x_out + p0 * MN, M, N, std::min(chunk, planes - p0), h, kh, kw, sc, iso,
                         maxit, static_cast<unsigned char*>(workspace), lay, Traj{}, red, pl.fwd);
    int rc2 = ln.finish();
    return rc ? rc : rc2;
}

// phases: 1 = forward recording the trajectory into the workspace (writes x_out), 2 = reverse sweep
// from a recorded workspace (x_out = that forward's output), 3 = both.  rec_flags (ADMM_REC_*): phase 1 alone
// records the extra h_bar trajectory only when asked (phase 2 must then be given h_bar).
int run_backward(int phases, int rec_flags, const float* y, const float* x_bar, float* y_bar, float* h_bar,
                 float* lambda_bar, float* rho_bar, int M, int N, int P, int B, const float* h, int kh, int kw,
                 const admm::ScalarSrc& sc, int iso, int maxit, float* x_out, void* workspace, size_t workspace_bytes,
                 void* stream, const admm_batch_reducer* reducer) {
    const admm_batch_reducer* red = (iso && reducer && reducer->fn) ? reducer : nullptr;
    if (h == nullptr) kh = kw = 0;
    int rc = check_shape(M, N, P, B, kh, kw, iso);
    if (rc) return rc;
    rc = check_common(y, x_out, maxit);
    if (rc) return rc;
    if ((phases & 2) && (reinterpret_cast<uintptr_t>(y_bar) & 15))
        return fail(ADMM_E_INVALID, "y_bar must be a 16-byte aligned device pointer (or NULL: not needed)");
    if ((phases & 2) && (!x_bar || (reinterpret_cast<uintptr_t>(x_bar) & 15)))
        return fail(ADMM_E_INVALID, "x_bar must be a 16-byte aligned device pointer");
    const size_t planes = (size_t)P * B;
    if (planes > 65535) return fail(ADMM_E_UNSUPPORTED, "the adjoint takes at most 65535 planes per call (split the batch)");
    // the plan (plan_paths): a replay (phase 2) is planned as the recording it replays was (its flags are in
    // the recording's tag; a replay whose options or arguments differ is rejected below)
    int pflags = rec_flags;
    if (phases == 2) {
        std::lock_guard<std::mutex> lk(g_rec_mu);
        auto it = g_rec.find(workspace);
        pflags = (h_bar != nullptr ? ADMM_REC_HBAR : 0) | (it != g_rec.end() && it->second.masks ? ADMM_REC_MASKS : 0);
    }
    // sharded (red): no plane-count rule, so that every shard records and sweeps in one layout (forward_impl)
    const PathPlan plan = plan_paths({M, N, iso != 0, kh > 0, phases == 3 ? ADMM_MODE_BACKWARD : ADMM_MODE_RECORD, pflags,
                                      h_bar != nullptr, rho_bar != nullptr, red ? 0 : planes});
    const bool want_h = plan.want_h;
    const bool ln_traj = plan.ln_traj;
    const bool use_masks = plan.masks;
    const bool iso_lane = plan.iso_lane;   // the fused isotropic sweep (no mask bits: s itself is needed)
    const BwdLayout bl = make_bwd_layout(M, N, planes, kh, kw, maxit, want_h, iso != 0, use_masks && !iso);
    rc = check_ws(workspace, workspace_bytes, bl.total);
    if (rc) return rc;
    RecTag tag = make_tag(M, N, P, B, kh, kw, iso, maxit, want_h, sc);
    tag.masks = use_masks;
    if (phases == 2) {
        std::lock_guard<std::mutex> lk(g_rec_mu);
        auto it = g_rec.find(workspace);
        if (it == g_rec.end())
            return fail(ADMM_E_INVALID, "workspace holds no recording (admm_tvd_forward_record_* first; a plain forward "
                                        "on the same workspace overwrites it)");
        if (!(it->second == tag))
            return fail(ADMM_E_INVALID, "replay does not match its recording (shape, PSF, iso, maxit, h_bar request, "
                                        "lambda / rho or library options changed between record and replay)");
        if (use_masks && rho_bar)
            return fail(ADMM_E_INVALID, "recorded with ADMM_REC_MASKS (soft-threshold branches only / the fused isotropic "
                                        "trajectory): rho_bar cannot be formed from it; record without the flag to get rho_bar");
        g_rec.erase(it);
    } else {
        std::lock_guard<std::mutex> lk(g_rec_mu);
        if (phases == 1) g_rec[workspace] = tag;
        else g_rec.erase(workspace);
    }
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
                                       nullptr, tr.m != nullptr, opt(ADMM_OPT_PLANE_STAGGER));
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

// ---- several branches of one shared input in one grid (Parallel(chcat, ...), net_build.jl:113-125) ----
// Workspace: per branch {tau, rho, lambda} (16 B each, one block), its C table and its lane-native tables;
// per grid plane the fused kernel's H^T y (= y) and s state, the trajectory (full s_k or mask bytes), the
// reverse sweep's sbar and Vsum state and the (rho_bar, tau_bar) partials.  After the forward, the H^T y
// slots hold each branch's Vsum (natural layout, y_bar only) and the s slots D x_K (rho_bar only).
struct MultiLayout {
    size_t prm, twM, twN, C, F, hln, sln, traj, sbar, vsl, part, rt, rtmp, total;
    size_t fmap, qpart, nrm, rmap;   // isotropic (ADMM_MULTI_ISO): f maps, q / R partials, |s| slots, R maps
};
constexpr int kMultiM = 256, kMultiN = 256;
size_t multi_C_bytes() { return align_up((size_t)(kMultiM / 2 + 1) * kMultiN * 4); }
size_t multi_F_bytes() { return align_up(admm::plane::tables_bytes()); }

// tau_bar partial rows of one branch's isotropic sweep: 512 per reverse step k = K .. 2 (iso_radj_kernel)
size_t multi_iso_rows(int K) { return (size_t)(K > 1 ? K - 1 : 1) * 512; }

MultiLayout make_multi_layout(size_t planes, int nbr, int maxit, int flags) {
    MultiLayout L{};
    size_t off = 0;
    auto take = [&](size_t bytes) {
        size_t o = off;
        off = align_up(off + bytes);
        return o;
    };
    const size_t MN = (size_t)kMultiM * kMultiN;
    const int K = maxit < 1 ? 1 : maxit;
    const bool rec = (flags & ADMM_MULTI_RECORD) != 0, iso = (flags & ADMM_MULTI_ISO) != 0;
    const bool masks = (flags & ADMM_REC_MASKS) != 0 && !iso;
    L.prm = take((size_t)nbr * 16);
    L.twM = take(kMultiM * 8);
    L.twN = take(kMultiN * 8);
    L.C = take((size_t)nbr * multi_C_bytes());
    L.F = take((size_t)nbr * multi_F_bytes());
    L.hln = take(planes * MN * 4);
    L.sln = take(planes * MN * 8);
    if (rec) {
        L.traj = take((size_t)(K > 1 ? K - 1 : 1) * planes * (masks ? MN / 2 : MN * 8));
        L.sbar = take(planes * MN * 8);
        L.vsl = take(planes * MN * 4);
        L.part = take(iso ? (size_t)nbr * multi_iso_rows(K) * 16 : planes * 16);
        L.rt = take((size_t)nbr * 16);
        L.rtmp = take((size_t)kRedParts * 2 * 8);
    }
    if (iso) {
        L.fmap = take((size_t)nbr * MN * 4);
        L.qpart = take(planes * MN * 4);
        if (rec) {
            L.nrm = take((size_t)(K > 1 ? K - 1 : 1) * nbr * MN * 4);
            L.rmap = take((size_t)nbr * MN * 4);
        }
    }
    L.total = off;
    return L;
}

int check_multi(int M, int N, int P, int B, int nbr, int maxit, int flags) {
    if (P < 1 || B < 1 || nbr < 1) return fail(ADMM_E_INVALID, "sizes must be positive (P=%d B=%d nbranch=%d)", P, B, nbr);
    if (maxit < 0) return fail(ADMM_E_INVALID, "maxit must be >= 0 (got %d)", maxit);
    if (flags & ~(ADMM_MULTI_RECORD | ADMM_REC_MASKS | ADMM_MULTI_ISO)) return fail(ADMM_E_INVALID, "unknown flags 0x%x", flags);
    if (M != kMultiM || N != kMultiN || !fused_enabled())
        return fail(ADMM_E_UNSUPPORTED, "the multi-branch solve is the fused 256 x 256 kernels (got %d x %d%s); "
                                        "solve the branches one by one", M, N, fused_enabled() ? "" : ", option FUSED = 0");
    if ((flags & ADMM_MULTI_ISO) && (flags & ADMM_MULTI_RECORD) && !fused_adj_enabled())
        return fail(ADMM_E_UNSUPPORTED, "an isotropic multi-branch recording needs the fused reverse sweep (option FUSED_ADJ)");
    if ((size_t)P * B * nbr > kChunkPlanes)
        return fail(ADMM_E_UNSUPPORTED, "at most %zu planes (nbranch * P * B) per multi-branch call", kChunkPlanes);
    return ADMM_OK;
}

admm::plane::Branches multi_branches(int P, int B, int nbr) {
    return admm::plane::Branches{P * B, nbr, P, (unsigned)(multi_F_bytes() / 4), 4u};
}

int forward_multi(const float* y, float* x_out, int M, int N, int P, int B, int nbr, const float* const* lambda,
                  const float* const* rho, int maxit, int flags, void* workspace, size_t workspace_bytes, void* stream) {
    int rc = check_multi(M, N, P, B, nbr, maxit, flags);
    if (rc) return rc;
    rc = check_common(y, x_out, maxit);
    if (rc) return rc;
    if (!lambda || !rho) return fail(ADMM_E_INVALID, "lambda and rho must be host arrays of nbranch device pointers");
    for (int i = 0; i < nbr; ++i)
        if (!lambda[i] || !rho[i]) return fail(ADMM_E_INVALID, "lambda[%d] / rho[%d] must be device pointers", i, i);
    const size_t planes = (size_t)P * B * nbr;
    const MultiLayout L = make_multi_layout(planes, nbr, maxit, flags);
    rc = check_ws(workspace, workspace_bytes, L.total);
    if (rc) return rc;
    {
        std::lock_guard<std::mutex> lk(g_rec_mu);
        g_rec.erase(workspace);
        if (flags & ADMM_MULTI_RECORD) {
            const int iso = (flags & ADMM_MULTI_ISO) != 0;
            RecTag t = make_tag(M, N, P, B, 0, 0, iso, maxit, false, admm::ScalarSrc{lambda[0], rho[0], 0.f, 0.f});
            t.nbr = nbr;
            t.masks = (flags & ADMM_REC_MASKS) != 0 || iso;   // no rho_bar from either
            g_rec[workspace] = t;
        }
    }
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
        rc = ln.run(ADMM_K_SETUP, [&] { return admm::plane::launch_tables(Ct, nullptr, F, s); });
        if (rc) return rc;
    }
    if (maxit == 0) {
        hipError_t e = hipMemsetAsync(x_out, 0, planes * (size_t)M * N * 4, s);
        if (e != hipSuccess) return fail(ADMM_E_HIP, "hipMemsetAsync: %s", hipGetErrorString(e));
        return ln.finish();
    }
    const admm::plane::Branches br = multi_branches(P, B, nbr);
    const bool rec = (flags & ADMM_MULTI_RECORD) != 0, masks = rec && (flags & ADMM_REC_MASKS) != 0;
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
                                         rec && !masks ? reinterpret_cast<float4*>(ws + L.traj) : nullptr,
                                         opt(ADMM_OPT_PLANE_STAGGER), &br,
                                         masks ? reinterpret_cast<unsigned*>(ws + L.traj) : nullptr);
    });
    if (rc) return rc;
    return ln.finish();
}

int backward_multi(const float* x_bar, float* y_bar, float* lambda_bar, float* rho_bar, int M, int N, int P, int B,
                   int nbr, int maxit, const float* x_out, void* workspace, size_t workspace_bytes, void* stream) {
    int rc = check_multi(M, N, P, B, nbr, maxit, 0);
    if (rc) return rc;
    if (!x_bar || !x_out || (reinterpret_cast<uintptr_t>(x_bar) & 15) || (reinterpret_cast<uintptr_t>(x_out) & 15) ||
        (reinterpret_cast<uintptr_t>(y_bar) & 15))
        return fail(ADMM_E_INVALID, "x_bar, x_out (and y_bar if given) must be 16-byte aligned device pointers");
    int flags = ADMM_MULTI_RECORD;
    {
        std::lock_guard<std::mutex> lk(g_rec_mu);
        auto it = g_rec.find(workspace);
        if (it == g_rec.end() || it->second.nbr != nbr)
            return fail(ADMM_E_INVALID, "workspace holds no multi-branch recording of %d branches "
                                        "(admm_tvd_forward_multi_dev_f32 with ADMM_MULTI_RECORD first)", nbr);
        const int iso = it->second.iso;
        RecTag t = make_tag(M, N, P, B, 0, 0, iso, maxit, false, admm::ScalarSrc{&g_dummy_scalar, &g_dummy_scalar, 0.f, 0.f});
        t.nbr = nbr;
        t.masks = it->second.masks;
        if (iso) flags |= ADMM_MULTI_ISO;
        if (!(it->second == t))
            return fail(ADMM_E_INVALID, "replay does not match its multi-branch recording (shape, maxit or library "
                                        "options changed)");
        if (t.masks && rho_bar)
            return fail(ADMM_E_INVALID, "recorded with ADMM_REC_MASKS (soft-threshold branches only) or ADMM_MULTI_ISO: "
                                        "rho_bar cannot be formed from it");
        if (t.masks) flags |= ADMM_REC_MASKS;
        g_rec.erase(it);
    }
    const size_t planes = (size_t)P * B * nbr, ppb = (size_t)P * B, MN = (size_t)M * N;
    const MultiLayout L = make_multi_layout(planes, nbr, maxit, flags);
    rc = check_ws(workspace, workspace_bytes, L.total);
    if (rc) return rc;
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
                                             prm, K, planes, s, &br, masks, opt(ADMM_OPT_PLANE_STAGGER));
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

}  // namespace

extern "C" {

int admm_tvd_forward_f32(const float* y, float* x_out, int M, int N, int P, int B, const float* h, int kh, int kw,
                         float lambda, float rho, int iso, int maxit, void* workspace, size_t workspace_bytes,
                         void* stream) {
    return admm_tvd_forward_sharded_f32(y, x_out, M, N, P, B, h, kh, kw, lambda, rho, iso, maxit, workspace,
                                        workspace_bytes, stream, nullptr);
}

int admm_tvd_forward_sharded_f32(const float* y, float* x_out, int M, int N, int P, int B, const float* h, int kh,
                                 int kw, float lambda, float rho, int iso, int maxit, void* workspace,
                                 size_t workspace_bytes, void* stream, const admm_batch_reducer* reducer) {
    int rc = check_lam_rho(lambda, rho);
    if (rc) return rc;
    return forward_impl(y, x_out, M, N, P, B, h, kh, kw, admm::ScalarSrc{nullptr, nullptr, lambda, rho}, iso, maxit,
                        workspace, workspace_bytes, stream, reducer);
}

int admm_tvd_forward_dev_f32(const float* y, float* x_out, int M, int N, int P, int B, const float* h, int kh, int kw,
                             const float* lambda, const float* rho, int iso, int maxit, void* workspace,
                             size_t workspace_bytes, void* stream, const admm_batch_reducer* reducer) {
    if (!lambda || !rho) return fail(ADMM_E_INVALID, "lambda and rho must be device pointers");
    return forward_impl(y, x_out, M, N, P, B, h, kh, kw, admm::ScalarSrc{lambda, rho, 0.f, 0.f}, iso, maxit,
                        workspace, workspace_bytes, stream, reducer);
}

int admm_tvd_backward_workspace_bytes(int M, int N, int P, int B, int kh, int kw, int iso, int maxit, int want_hbar,
                                      size_t* out_bytes) {
    if (!out_bytes) return fail(ADMM_E_INVALID, "out_bytes is NULL");
    int rc = check_shape(M, N, P, B, kh, kw, iso);
    if (rc) return rc;
    if (maxit < 0) return fail(ADMM_E_INVALID, "maxit must be >= 0");
    if ((size_t)P * B > 65535) return fail(ADMM_E_UNSUPPORTED, "the adjoint takes at most 65535 planes per call (split the batch)");
    const PathPlan pl = plan_paths({M, N, iso != 0, kh > 0, ADMM_MODE_RECORD, want_hbar, false, false, (size_t)P * B});
    *out_bytes = make_bwd_layout(M, N, (size_t)P * B, kh, kw, maxit, pl.want_h, iso != 0, pl.masks && !iso).total;
    return ADMM_OK;
}

int admm_tvd_backward_f32(const float* y, const float* x_bar, float* y_bar, float* h_bar, float* lambda_bar,
                          float* rho_bar, int M, int N, int P, int B, const float* h, int kh, int kw, float lambda,
                          float rho, int iso, int maxit, float* x_out, void* workspace, size_t workspace_bytes,
                          void* stream) {
    return admm_tvd_backward_sharded_f32(y, x_bar, y_bar, h_bar, lambda_bar, rho_bar, M, N, P, B, h, kh, kw, lambda,
                                         rho, iso, maxit, x_out, workspace, workspace_bytes, stream, nullptr);
}

int admm_tvd_backward_sharded_f32(const float* y, const float* x_bar, float* y_bar, float* h_bar, float* lambda_bar,
                                  float* rho_bar, int M, int N, int P, int B, const float* h, int kh, int kw,
                                  float lambda, float rho, int iso, int maxit, float* x_out, void* workspace,
                                  size_t workspace_bytes, void* stream, const admm_batch_reducer* reducer) {
    int rc = check_lam_rho(lambda, rho);
    if (rc) return rc;
    return run_backward(3, 0, y, x_bar, y_bar, h_bar, lambda_bar, rho_bar, M, N, P, B, h, kh, kw,
                        admm::ScalarSrc{nullptr, nullptr, lambda, rho}, iso, maxit, x_out, workspace, workspace_bytes,
                        stream, reducer);
}

int admm_tvd_backward_dev_f32(const float* y, const float* x_bar, float* y_bar, float* h_bar, float* lambda_bar,
                              float* rho_bar, int M, int N, int P, int B, const float* h, int kh, int kw,
                              const float* lambda, const float* rho, int iso, int maxit, float* x_out, void* workspace,
                              size_t workspace_bytes, void* stream, const admm_batch_reducer* reducer) {
    if (!lambda || !rho) return fail(ADMM_E_INVALID, "lambda and rho must be device pointers");
    return run_backward(3, 0, y, x_bar, y_bar, h_bar, lambda_bar, rho_bar, M, N, P, B, h, kh, kw,
                        admm::ScalarSrc{lambda, rho, 0.f, 0.f}, iso, maxit, x_out, workspace, workspace_bytes, stream,
                        reducer);
}

int admm_tvd_forward_record_f32(const float* y, float* x_out, int M, int N, int P, int B, const float* h, int kh,
                                int kw, float lambda, float rho, int iso, int maxit, int want_hbar, void* workspace,
                                size_t workspace_bytes, void* stream, const admm_batch_reducer* reducer) {
    int rc = check_lam_rho(lambda, rho);
    if (rc) return rc;
    return run_backward(1, want_hbar, y, nullptr, nullptr, nullptr, nullptr, nullptr, M, N, P, B, h, kh, kw,
                        admm::ScalarSrc{nullptr, nullptr, lambda, rho}, iso, maxit, x_out, workspace, workspace_bytes,
                        stream, reducer);
}

int admm_tvd_forward_record_dev_f32(const float* y, float* x_out, int M, int N, int P, int B, const float* h, int kh,
                                    int kw, const float* lambda, const float* rho, int iso, int maxit, int want_hbar,
                                    void* workspace, size_t workspace_bytes, void* stream,
                                    const admm_batch_reducer* reducer) {
    if (!lambda || !rho) return fail(ADMM_E_INVALID, "lambda and rho must be device pointers");
    return run_backward(1, want_hbar, y, nullptr, nullptr, nullptr, nullptr, nullptr, M, N, P, B, h, kh, kw,
                        admm::ScalarSrc{lambda, rho, 0.f, 0.f}, iso, maxit, x_out, workspace, workspace_bytes, stream,
                        reducer);
}

int admm_tvd_backward_recorded_f32(const float* y, const float* x_bar, float* y_bar, float* h_bar, float* lambda_bar,
                                   float* rho_bar, int M, int N, int P, int B, const float* h, int kh, int kw,
                                   float lambda, float rho, int iso, int maxit, const float* x_out, void* workspace,
                                   size_t workspace_bytes, void* stream, const admm_batch_reducer* reducer) {
    int rc = check_lam_rho(lambda, rho);
    if (rc) return rc;
    return run_backward(2, 0, y, x_bar, y_bar, h_bar, lambda_bar, rho_bar, M, N, P, B, h, kh, kw,
                        admm::ScalarSrc{nullptr, nullptr, lambda, rho}, iso, maxit, const_cast<float*>(x_out),
                        workspace, workspace_bytes, stream, reducer);
}

int admm_tvd_backward_recorded_dev_f32(const float* y, const float* x_bar, float* y_bar, float* h_bar,
                                       float* lambda_bar, float* rho_bar, int M, int N, int P, int B, const float* h,
                                       int kh, int kw, const float* lambda, const float* rho, int iso, int maxit,
                                       const float* x_out, void* workspace, size_t workspace_bytes, void* stream,
                                       const admm_batch_reducer* reducer) {
    if (!lambda || !rho) return fail(ADMM_E_INVALID, "lambda and rho must be device pointers");
    return run_backward(2, 0, y, x_bar, y_bar, h_bar, lambda_bar, rho_bar, M, N, P, B, h, kh, kw,
                        admm::ScalarSrc{lambda, rho, 0.f, 0.f}, iso, maxit, const_cast<float*>(x_out), workspace,
                        workspace_bytes, stream, reducer);
}

int admm_set_option(int option, int value) {
    if (option < 0 || option >= ADMM_OPT_COUNT) return fail(ADMM_E_INVALID, "unknown option %d", option);
    g_opt[option].store(value, std::memory_order_relaxed);
    return ADMM_OK;
}

int admm_get_option(int option, int* value) {
    if (option < 0 || option >= ADMM_OPT_COUNT || !value) return fail(ADMM_E_INVALID, "bad option query %d", option);
    *value = opt(option);
    return ADMM_OK;
}

int admm_profile_enable(int on) {
    g_prof.on = on != 0;
    return ADMM_OK;
}

int admm_profile_reset(void) {
    std::lock_guard<std::mutex> lk(g_prof.mu);
    for (int i = 0; i < ADMM_K_COUNT; ++i) {
        g_prof.ms[i] = 0.0;
        g_prof.n[i] = 0;
    }
    return ADMM_OK;
}

int admm_profile_get(int kernel_class, double* total_ms, long long* launches) {
    if (kernel_class < 0 || kernel_class >= ADMM_K_COUNT || !total_ms || !launches)
        return fail(ADMM_E_INVALID, "bad profile query");
    std::lock_guard<std::mutex> lk(g_prof.mu);
    *total_ms = g_prof.ms[kernel_class];
    *launches = g_prof.n[kernel_class];
    return ADMM_OK;
}

int admm_query_paths(int M, int N, int iso, int kh, long long planes, int mode, int flags, int want_hbar, int want_rho,
                     int* fwd_path, int* bwd_path) {
    if (!fwd_path || !bwd_path) return fail(ADMM_E_INVALID, "admm_query_paths: NULL output");
    if (mode != ADMM_MODE_FORWARD && mode != ADMM_MODE_RECORD && mode != ADMM_MODE_BACKWARD)
        return fail(ADMM_E_INVALID, "admm_query_paths: unknown mode %d", mode);
    const int rc = check_shape(M, N, 1, 1, kh, kh, iso);
    if (rc) return rc;
    if (planes < 0) return fail(ADMM_E_INVALID, "admm_query_paths: planes must be >= 0");
    const PathPlan pl = plan_paths({M, N, iso != 0, kh > 0, mode, flags, want_hbar != 0, want_rho != 0, (size_t)planes});
    *fwd_path = pl.fwd;
    *bwd_path = pl.bwd;
    return ADMM_OK;
}

const char* admm_path_name(int path) {
    switch (path) {
        case ADMM_PATH_FUSED: return "fused";
        case ADMM_PATH_FUSED_ISO: return "fused_iso";
        case ADMM_PATH_2PASS: return "2pass";
        case ADMM_PATH_2PASS_ISO: return "2pass_iso";
        case ADMM_PATH_RESIDENT: return "resident";
        case ADMM_PATH_SMOOTH: return "smooth";
        case ADMM_PATH_RUNTIME: return "runtime";
        case ADMM_PATH_SWEEP_FUSED: return "sweep_fused";
        case ADMM_PATH_SWEEP_FUSED_ISO: return "sweep_fused_iso";
        case ADMM_PATH_SWEEP_2PASS: return "sweep_2pass";
        case ADMM_PATH_SWEEP_2PASS_ISO: return "sweep_2pass_iso";
        case ADMM_PATH_SWEEP_RUNTIME: return "sweep_runtime";
        case ADMM_PATH_SWEEP_RUNTIME_ISO: return "sweep_runtime_iso";
        case ADMM_PATH_RESIDENT_ISO: return "resident_iso";
        default: return "none";
    }
}

int admm_copy_async(void* dst, const void* src, size_t bytes, void* stream) {
    if (bytes == 0) return ADMM_OK;
    if (!dst || !src) return fail(ADMM_E_INVALID, "admm_copy_async: NULL pointer");
    const hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(ADMM_E_HIP, "admm_copy_async: %s", hipGetErrorString(e));
    return ADMM_OK;
}

static_assert(sizeof(hipIpcMemHandle_t) == ADMM_IPC_HANDLE_BYTES, "hipIpcMemHandle_t size");

int admm_ipc_get_handle(const void* dev_ptr, void* handle_out, size_t* offset_out) {
    if (!dev_ptr || !handle_out || !offset_out) return fail(ADMM_E_INVALID, "admm_ipc_get_handle: NULL pointer");
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    hipError_t e = hipMemGetAddressRange(&base, &size, const_cast<void*>(dev_ptr));
    if (e != hipSuccess) return fail(ADMM_E_HIP, "admm_ipc_get_handle: hipMemGetAddressRange: %s", hipGetErrorString(e));
    hipIpcMemHandle_t h;
    e = hipIpcGetMemHandle(&h, base);
    if (e != hipSuccess) return fail(ADMM_E_HIP, "admm_ipc_get_handle: hipIpcGetMemHandle: %s", hipGetErrorString(e));
    std::memcpy(handle_out, &h, sizeof(h));
    *offset_out = static_cast<size_t>(static_cast<const char*>(dev_ptr) - static_cast<const char*>(base));
    return ADMM_OK;
}

int admm_ipc_open(const void* handle, int device, void** dev_ptr_out) {
    if (!handle || !dev_ptr_out) return fail(ADMM_E_INVALID, "admm_ipc_open: NULL pointer");
    int prev = -1;
    hipError_t e = hipGetDevice(&prev);
    if (e == hipSuccess && prev != device) e = hipSetDevice(device);
    if (e != hipSuccess) return fail(ADMM_E_HIP, "admm_ipc_open: select device %d: %s", device, hipGetErrorString(e));
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle, sizeof(h));
    void* p = nullptr;
    e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
    if (prev != device) (void)hipSetDevice(prev);
    if (e != hipSuccess) return fail(ADMM_E_HIP, "admm_ipc_open: hipIpcOpenMemHandle on device %d: %s", device, hipGetErrorString(e));
    *dev_ptr_out = p;
    return ADMM_OK;
}

int admm_ipc_close(void* dev_ptr, int device) {
    if (!dev_ptr) return fail(ADMM_E_INVALID, "admm_ipc_close: NULL pointer");
    int prev = -1;
    hipError_t e = hipGetDevice(&prev);
    if (e == hipSuccess && prev != device) e = hipSetDevice(device);
    if (e != hipSuccess) return fail(ADMM_E_HIP, "admm_ipc_close: select device %d: %s", device, hipGetErrorString(e));
    e = hipIpcCloseMemHandle(dev_ptr);
    if (prev != device) (void)hipSetDevice(prev);
    if (e != hipSuccess) return fail(ADMM_E_HIP, "admm_ipc_close: %s", hipGetErrorString(e));
    return ADMM_OK;
}

int admm_tvd_multi_workspace_bytes(int M, int N, int P, int B, int nbranch, int maxit, int flags, size_t* out_bytes) {
    if (!out_bytes) return fail(ADMM_E_INVALID, "out_bytes is NULL");
    int rc = check_multi(M, N, P, B, nbranch, maxit, flags);
    if (rc) return rc;
    *out_bytes = make_multi_layout((size_t)P * B * nbranch, nbranch, maxit, flags).total;
    return ADMM_OK;
}

int admm_tvd_forward_multi_dev_f32(const float* y, float* x_out, int M, int N, int P, int B, int nbranch,
                                   const float* const* lambda, const float* const* rho, int maxit, int flags,
                                   void* workspace, size_t workspace_bytes, void* stream) {
    return forward_multi(y, x_out, M, N, P, B, nbranch, lambda, rho, maxit, flags, workspace, workspace_bytes, stream);
}

int admm_tvd_backward_multi_recorded_dev_f32(const float* x_bar, float* y_bar, float* lambda_bar, float* rho_bar, int M,
                                             int N, int P, int B, int nbranch, int maxit, const float* x_out,
                                             void* workspace, size_t workspace_bytes, void* stream) {
    return backward_multi(x_bar, y_bar, lambda_bar, rho_bar, M, N, P, B, nbranch, maxit, x_out, workspace,
                          workspace_bytes, stream);
}

}  // extern "C"
