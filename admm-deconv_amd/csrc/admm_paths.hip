// admm_paths.hip -- the path decision table and the library options (host code only; see capi_internal.hpp).
// Which kernels a call runs is decided in plan_paths and nowhere else; admm_launch.hip executes the plan and
// admm_query_paths returns it to tests without a GPU.  The tile-size policy of the 2-pass and runtime-length
// kernels lives here too: the workspace layouts (admm_capi.hip) and the launches (admm_launch.hip) share it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>

#include "capi_internal.hpp"
#include "fft_reg.hpp"
#include "resident_api.hpp"
#include "smooth_api.hpp"

namespace admm_capi {

// Library options (admm_set_option; process-global, read at each call).  The defaults are the tuned
// choices; the others exist for tests (fused vs 2-pass) and tuning experiments.  A recording stores
// the option values it was made with, and its replay rejects a change (RecTag below).
std::atomic<int> g_opt[ADMM_OPT_COUNT] = {{1}, {1}, {0}, {0}, {0}, {0}, {0}, {1}, {1}, {-1}, {4}};
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
    if (v == 256 || ((v == 512 || v == 1024) && N >= 256)) nt = v;
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
// MALL-resident schedule (ADMM_OPT_MALL_STREAMS; DESIGN.md s5 "Round 6, c4").  A 2-pass iteration touches
// 28 B/px (packed spectrum in and out 8, s in and out 16, Y_h 4): at c4 (768 planes of 512^2) 5.6 GB per
// iteration, so every pass streams from HBM.  Chunks of ~224 MiB / n (8 planes at 512^2, n = 4) run all K
// iterations with n of them in flight: their sets stay in the 256 MiB Infinity Cache, and the n streams overlap
// each other's kernel tails.  tools/c4_chunk_probe.py, profiles/r06_c4_chunk_probe.jsonl: 81.8 -> 75.7 ms per c4
// solve (8 planes x 4 streams; 16 x 2 77.2, 8 x 2 97.8: one or two small grids alone leave the chip idle; 5-12
// streams 97-149 ms, profiles/r06_c4_mall_streams_sweep.txt -- their 4-5 plane chunks are too small: 4 x 4 97.0,
// 5 x 4 85.3 ms; with 8 hardware queues 6 / 8 streams are slower still, profiles/r06_c4_hw_queues_probe.txt).
// The smooth-length 2-pass kernels gain the same way (480 x 640 x 64 / 256 +5 / +7 %, 384^2 x 512 +11 %).
ChunkPlan forward_chunks(int M, int N, size_t planes, bool iso, int fwd_path) {
    const size_t base = chunk_planes(planes, iso);
    const int n = opt(ADMM_OPT_MALL_STREAMS);
    const bool two_pass = fwd_path == ADMM_PATH_2PASS || fwd_path == ADMM_PATH_SMOOTH || fwd_path == ADMM_PATH_RUNTIME;
    if (iso || n <= 1 || !two_pass) return {base, 1};
    constexpr size_t kMall = size_t(256) << 20, kBudget = size_t(224) << 20;
    const size_t per_plane = 28 * (size_t)M * N;
    if (planes * per_plane <= 2 * kMall) return {base, 1};
    size_t chunk = kBudget / ((size_t)n * per_plane);
    // chunks of 1-2 large planes lose (2048^2 x 8: 1-plane chunks -15 %, 1000^2 x 64: 2-plane chunks -2 %;
    // profiles/r06_mall_generic_ab.jsonl): whole batch
    if (chunk < 4) return {base, 1};
    if (chunk > base) chunk = base;
    return {chunk, n > 16 ? 16 : n};
}

// Several 256 x 256 branches in one grid (admm_tvd_forward_multi_dev_f32): the per-plane kernels from the fused
// paths' plane counts in all (kMinFused / kMinFusedIso), below them the 2-pass kernels over every branch's planes
// (the c5 training step at batch 2 has 30: tools/small_batch_probe.py, profiles/r05_small_batch_probe.jsonl).
bool multi_two_pass(size_t planes, int flags) {
    const bool iso = (flags & ADMM_MULTI_ISO) != 0;
    return !enough_planes(PathIn{kMultiM, kMultiN, iso, false, ADMM_MODE_FORWARD, 0, false, false, planes},
                          iso ? kMinFusedIso : kMinFused);
}
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

}  // namespace admm_capi

using namespace admm_capi;

extern "C" {

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

int admm_query_forward_schedule(int M, int N, int iso, int kh, long long planes, long long* chunk_planes,
                                int* streams) {
    if (!chunk_planes || !streams) return fail(ADMM_E_INVALID, "admm_query_forward_schedule: NULL output");
    const int rc = check_shape(M, N, 1, 1, kh, kh, iso);
    if (rc) return rc;
    if (planes <= 0) return fail(ADMM_E_INVALID, "admm_query_forward_schedule: planes must be > 0");
    const PathPlan pl = plan_paths({M, N, iso != 0, kh > 0, ADMM_MODE_FORWARD, 0, false, false, (size_t)planes});
    const ChunkPlan cp = forward_chunks(M, N, (size_t)planes, iso != 0, pl.fwd);
    *chunk_planes = (long long)std::min(cp.chunk, (size_t)planes);
    *streams = cp.streams;
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

}  // extern "C"
