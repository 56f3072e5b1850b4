// capi_internal.hpp -- declarations shared by the library's host translation units:
//   admm_capi.hip   the extern "C" ABI (include/admm_deconv.h): argument validation, workspace layouts and
//                   queries, the recordings registry, the profiler API, the output transport (copy / IPC)
//   admm_paths.hip  the path decision table (plan_paths), the library options and the tile-size policy
//   admm_launch.hip launch sequencing of the 2-pass / runtime-length / CU-resident / fused paths (the only TU
//                   that includes the 2-pass kernels)
// Reference interface: tvd_fft / tvd_fft_gpu, /root/reference/src/ops/ops.jl:99-188.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <mutex>
#include <type_traits>
#include <vector>

#include "../../include/admm_deconv.h"
#include "layout.hpp"
#include "plane_api.hpp"
#include "scalar_src.hpp"

namespace admm_capi {

using namespace admm::layout;
constexpr int kGenMax = 4096;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

// ---- options and tile policy (admm_paths.hip) ----
int opt(int k);
bool fused_enabled();
bool fused_adj_enabled();
int line_T(int M, int N);
size_t line_lds(int M, int T);
size_t fwdinv_lds(int M, int T);
int column_threads(int N);
int column_KB(int M, int N);
int bwd_line_T(int M, int N, bool iso);
size_t column_lds(int N, int KB);
size_t iso_a_lds(int M, int T);
size_t iso_b_lds(int M, int T);
int gen_T(int M, int N);
int gen_nb(int N, int T);
int gen_KB(int M, int N);
size_t gen_lds_line(int M, int T, bool upd);
size_t gen_lds_col(int N, int KB);

// ---- profiler (admm_capi.hip owns g_prof) ----
struct Prof {
    bool on = false;
    double ms[ADMM_K_COUNT] = {};
    long long n[ADMM_K_COUNT] = {};
    std::mutex mu;
};
extern Prof g_prof;

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

int check_shape(int M, int N, int P, int B, int kh, int kw, int iso);

// Planes per launch sequence.  The 2-pass kernels index planes by blockIdx.y (<= 65535), so a larger
// anisotropic forward runs as consecutive chunks of this many planes through one chunk-sized workspace
// (planes are independent, ops.jl:168-173).  A multiple of 256: every chunk but the last fills whole
// waves of the fused kernel (one workgroup per CU).
constexpr size_t kChunkPlanes = 255 * 256;
inline size_t launch_planes(size_t planes) { return planes < kChunkPlanes ? planes : kChunkPlanes; }
// The isotropic prox couples the whole batch through the per-pixel norm (ops.jl:6), so an isotropic
// batch is never split: it runs as one launch sequence of up to 65535 planes (check_shape's limit).
inline size_t chunk_planes(size_t planes, bool iso) { return iso ? planes : launch_planes(planes); }

// MALL-resident schedule of the anisotropic 2-pass forward (ADMM_OPT_MALL_STREAMS, DESIGN.md s5 "Round 6, c4"):
// planes in chunks of `chunk`, `streams` chunks in flight (the caller's stream + library streams), each chunk's
// per-iteration working set kept in the 256 MiB Infinity Cache.  streams = 1: the plain chunking above.
struct ChunkPlan {
    size_t chunk;
    int streams;
};
ChunkPlan forward_chunks(int M, int N, size_t planes, bool iso, int fwd_path);
// the library's own streams on the current device (created once; non-blocking)
hipStream_t lib_stream(int i);
struct PathPlan;
// forward workspace bytes (one chunk layout, or one per stream of the MALL-resident schedule)
size_t forward_ws_bytes(int M, int N, size_t planes, int kh, bool iso, const PathPlan* pl = nullptr);

// Trajectory recorded by the forward for the backward (all optional).
struct Traj {
    float* s = nullptr;      // (K-1) x planes x 2 x M x N : s_k for k = 1..K-1
    float2* v = nullptr;     // K x planes x N x M/2        : forward dim-2 spectra (h_bar only)
    double2* sig = nullptr;  // (M/2+1) x N                 : top-left PSF spectrum (h_bar only)
    float* nrm = nullptr;    // (K-1) x M x N               : isotropic batch norm of s_k (iso only)
    unsigned* m = nullptr;   // (K-1) x planes x 16 x 512   : ST mask bytes of s_k instead of s (fused only)
    bool iso_lane = false;   // isotropic 256 x 256: s and nrm lane-native (plane_iso.hip), for the fused adjoint
};

// ---- path selection (admm_paths.hip) ----
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
enum MinPlanesFor { kMinFused, kMinFusedIso, kMinResident, kMinResidentIso };
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
PathPlan plan_paths(const PathIn& q);

// ---- backward workspace (admm_capi.hip) ----
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
                          bool masks = false);

// ---- several branches in one grid (admm_capi.hip) ----
// Workspace: per branch {tau, rho, lambda} (16 B each, one block), its C table and its lane-native tables;
// per grid plane the fused kernel's H^T y (= y) and s state, the trajectory (full s_k or mask bytes), the
// reverse sweep's sbar and Vsum state and the (rho_bar, tau_bar) partials.  After the forward, the H^T y
// slots hold each branch's Vsum (natural layout, y_bar only) and the s slots D x_K (rho_bar only).
struct MultiLayout {
    size_t prm, twM, twN, C, F, hln, sln, traj, sbar, vsl, part, rt, rtmp, total;
    size_t fmap, qpart, nrm, rmap;   // isotropic (ADMM_MULTI_ISO): f maps, q / R partials, |s| slots, R maps
    // Below the plane-count rule the branches run the 2-pass kernels in one grid (multi_two_pass): spectra, s
    // state (anisotropic: sA / sbA ping-pong), and for the reverse sweep sbar (two), Vsum and (isotropic) vbar and
    // the plane-group R partials; qpart then holds the plane-group |s|^2 partials, traj / nrm the natural-layout
    // s_k / |s_k| slots (|s_k| per branch), part the (rho_bar, tau_bar) rows of every branch (pbs doubles apart,
    // rows_b per step)
    bool two_pass;
    size_t spec0, spec1, sA, sbA, sbB, vsum, wbar, Rpart, pbs;
    int ngb, G, rows_b, nblk_a;
};
constexpr int kMultiM = 256, kMultiN = 256;
// several branches below the fused kernels' plane-count rule run the 2-pass kernels (admm_paths.hip)
bool multi_two_pass(size_t planes, int flags);
size_t multi_C_bytes();
size_t multi_F_bytes();
size_t multi_iso_rows(int K);
admm::plane::Branches multi_branches(int P, int B, int nbr);

// ---- launch sequencing (admm_launch.hip) ----
// tables = false: the workspace already holds this call's twiddles, C / G tables and scalar block (a later plane
// chunk of the same call through the same chunk workspace): the setup kernels are not launched again
int run_forward(Launcher& ln, const float* y, float* x_out, int M, int N, size_t planes, const float* h, int kh,
                int kw, const admm::ScalarSrc& sc, int iso, int maxit, unsigned char* ws, const Layout& lay,
                const Traj& tr, const admm_batch_reducer* red, int fwd_path, bool tables = true);
// everything run_backward does after validating the call and updating the recordings registry
int launch_backward(int phases, const float* y, const float* x_bar, float* y_bar, float* h_bar, float* lambda_bar,
                    float* rho_bar, int M, int N, size_t planes, const float* h, int kh, int kw,
                    const admm::ScalarSrc& sc, int iso, int maxit, float* x_out, void* workspace, void* stream,
                    const admm_batch_reducer* red, const PathPlan& plan, const BwdLayout& bl);
int launch_forward_multi(const float* y, float* x_out, int M, int N, int P, int B, int nbr, const float* const* lambda,
                         const float* const* rho, int maxit, int flags, void* workspace, void* stream, size_t planes,
                         const MultiLayout& L);
int launch_backward_multi(const float* x_bar, float* y_bar, float* lambda_bar, float* rho_bar, int M, int N, int P,
                          int B, int nbr, int maxit, const float* x_out, void* workspace, void* stream, int flags,
                          size_t planes, size_t ppb, size_t MN, const MultiLayout& L);

}  // namespace admm_capi
