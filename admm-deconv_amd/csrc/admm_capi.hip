// admm_capi.hip -- extern "C" boundary (include/admm_deconv.h) for the ADMM TV-deconvolution
// solve on MI355X.  Replaces tvd_fft / tvd_fft_gpu (/root/reference/src/ops/ops.jl:99-188).
//
// This translation unit is the ABI: it validates every call, carves and queries the caller's workspace,
// keeps the recordings registry (a replay must match its recording) and the profiler, and hands the call
// to the launch sequencing (admm_launch.hip) with the plan of the path table (admm_paths.hip).  Nothing is
// allocated and nothing synchronises unless the optional profiler is on.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <mutex>
#include <unordered_map>
#include <string>

#include "capi_internal.hpp"

namespace admm {
// admm_clamp_backward_f32: four elements per thread (16-B accesses when the three pointers allow), grid-strided
__global__ __launch_bounds__(256) void clamp_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                        float* dx, size_t n, float lo, float hi) {
    const bool vec = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(dx)) &
                      15) == 0;
    for (size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += (size_t)gridDim.x * 256 * 4) {
        if (vec && i + 4 <= n) {
            const float4 a = *reinterpret_cast<const float4*>(x + i);
            const float4 g = *reinterpret_cast<const float4*>(dy + i);
            float4 r;
            r.x = (a.x >= lo && a.x <= hi) ? g.x : 0.0f;
            r.y = (a.y >= lo && a.y <= hi) ? g.y : 0.0f;
            r.z = (a.z >= lo && a.z <= hi) ? g.z : 0.0f;
            r.w = (a.w >= lo && a.w <= hi) ? g.w : 0.0f;
            *reinterpret_cast<float4*>(dx + i) = r;
        } else {
            for (size_t j = i; j < i + 4 && j < n; ++j) dx[j] = (x[j] >= lo && x[j] <= hi) ? dy[j] : 0.0f;
        }
    }
}
}  // namespace admm

namespace admm_capi {

thread_local std::string g_err;
Prof g_prof;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

}  // namespace admm_capi

namespace admm_internal {
// error reporting for the other translation units of the library (metrics_capi.hip)
int fail_msg(int code, const char* msg) {
    admm_capi::g_err = msg;
    return code;
}
}  // namespace admm_internal

namespace admm_capi {

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

}  // namespace admm_capi

using namespace admm_capi;

extern "C" {

int admm_abi_version(void) { return ADMM_ABI_VERSION; }

const char* admm_last_error(void) { return g_err.c_str(); }

int admm_tvd_workspace_bytes(int M, int N, int P, int B, int kh, int kw, int iso, size_t* out_bytes) {
    if (!out_bytes) return fail(ADMM_E_INVALID, "out_bytes is NULL");
    int rc = check_shape(M, N, P, B, kh, kw, iso);
    if (rc) return rc;
    *out_bytes = forward_ws_bytes(M, N, (size_t)P * B, kh, iso != 0);
    return ADMM_OK;
}

}  // extern "C"

namespace admm_capi {

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

BwdLayout make_bwd_layout(int M, int N, size_t planes, int kh, int kw, int maxit, bool want_h, bool iso,
                          bool masks) {
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
    int sharded; // recorded with a batch reducer: sharded calls plan without the plane-count rule, so a replay
                 // with (or without) one must match or it could plan another sweep than the trajectory's layout
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

// Library streams of the MALL-resident schedule: created once per device, never destroyed (non-blocking; the
// forward orders them against the caller's stream with events).
hipStream_t lib_stream(int i) {
    static std::mutex mu;
    static std::vector<std::vector<hipStream_t>> pool;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    if ((int)pool.size() <= dev) pool.resize(dev + 1);
    auto& v = pool[dev];
    while ((int)v.size() <= i) {
        hipStream_t st = nullptr;
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return nullptr;
        v.push_back(st);
    }
    return v[i];
}

// forward workspace: one chunk layout, or one per stream of the MALL-resident schedule
size_t forward_ws_bytes(int M, int N, size_t planes, int kh, bool iso, const PathPlan* plp) {
    const PathPlan pl = plp ? *plp : plan_paths({M, N, iso, kh > 0, ADMM_MODE_FORWARD, 0, false, false, planes});
    const ChunkPlan cp = forward_chunks(M, N, planes, iso, pl.fwd);
    const size_t one = make_layout(M, N, cp.chunk, kh > 0, iso).total;
    return cp.streams > 1 ? (size_t)cp.streams * align_up(one) : one;
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
    // a sharded isotropic solve plans without the plane-count rule: every shard must take the same path, since
    // the fused and 2-pass kernels hand the reducer their sum maps in different layouts (lane-native float2 vs
    // natural), and uneven shards can fall on either side of a threshold
    const PathPlan pl = plan_paths({M, N, iso != 0, kh > 0, ADMM_MODE_FORWARD, 0, false, false, red ? 0 : planes});
    const ChunkPlan cp = forward_chunks(M, N, planes, iso != 0, pl.fwd);
    const size_t chunk = cp.chunk;   // an isotropic batch is one chunk
    const Layout lay = make_layout(M, N, chunk, kh > 0, iso != 0);
    rc = check_ws(workspace, workspace_bytes, forward_ws_bytes(M, N, planes, kh, iso != 0, &pl));
    if (rc) return rc;
    rec_forget(workspace);   // whatever was recorded there is overwritten now
    const hipStream_t s0 = reinterpret_cast<hipStream_t>(stream);
    const size_t MN = (size_t)M * N;
    unsigned char* ws = static_cast<unsigned char*>(workspace);
    if (cp.streams <= 1) {
        Launcher ln{s0, g_prof.on, {}};
        // the tables (twiddles, C / G, scalars) once: later chunks reuse them from the same workspace
        for (size_t p0 = 0; p0 < planes && rc == 0; p0 += chunk)
            rc = run_forward(ln, y + p0 * MN, x_out + p0 * MN, M, N, std::min(chunk, planes - p0), h, kh, kw, sc, iso,
                             maxit, ws, lay, Traj{}, red, pl.fwd, p0 == 0);
        int rc2 = ln.finish();
        return rc ? rc : rc2;
    }
    // MALL-resident schedule: chunk i on stream i mod n (the caller's stream and n - 1 library streams), each stream
    // with its own chunk workspace; fork and join through events on the caller's stream
    const int n = cp.streams;
    const size_t stride = align_up(lay.total);
    std::vector<Launcher> lns;
    lns.reserve(n);
    lns.push_back(Launcher{s0, g_prof.on, {}});
    hipEvent_t fork = nullptr;
    if (hipEventCreateWithFlags(&fork, hipEventDisableTiming) != hipSuccess || hipEventRecord(fork, s0) != hipSuccess)
        return fail(ADMM_E_HIP, "MALL schedule: fork event");
    for (int k = 1; k < n; ++k) {
        hipStream_t sk = lib_stream(k - 1);
        if (!sk || hipStreamWaitEvent(sk, fork, 0) != hipSuccess) {
            hipEventDestroy(fork);
            return fail(ADMM_E_HIP, "MALL schedule: library stream %d", k);
        }
        lns.push_back(Launcher{sk, g_prof.on, {}});
    }
    hipEventDestroy(fork);   // (released once the waits have consumed it)
    size_t i = 0;
    for (size_t p0 = 0; p0 < planes && rc == 0; p0 += chunk, ++i) {
        const int k = (int)(i % (size_t)n);
        // each stream's chunk workspace builds the tables with its first chunk (96 setup launches per c4 solve -> 4)
        rc = run_forward(lns[k], y + p0 * MN, x_out + p0 * MN, M, N, std::min(chunk, planes - p0), h, kh, kw, sc, iso,
                         maxit, ws + (size_t)k * stride, lay, Traj{}, red, pl.fwd, i < (size_t)n);
    }
    // join: the caller's stream waits for every library stream (also after an error, so nothing is left running
    // against the caller's buffers unordered)
    for (int k = 1; k < n; ++k) {
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess) {
            if (hipEventRecord(e, lns[k].s) != hipSuccess || hipStreamWaitEvent(s0, e, 0) != hipSuccess)
                rc = rc ? rc : fail(ADMM_E_HIP, "MALL schedule: join");
            hipEventDestroy(e);
        } else if (!rc) {
            rc = fail(ADMM_E_HIP, "MALL schedule: join event");
        }
    }
    for (auto& l : lns) {
        const int r2 = l.finish();
        if (!rc) rc = r2;
    }
    return rc;
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
    tag.sharded = red != nullptr;
    if (phases == 2) {
        std::lock_guard<std::mutex> lk(g_rec_mu);
        auto it = g_rec.find(workspace);
        if (it == g_rec.end())
            return fail(ADMM_E_INVALID, "workspace holds no recording (admm_tvd_forward_record_* first; a plain forward "
                                        "on the same workspace overwrites it)");
        if (!(it->second == tag))
            return fail(ADMM_E_INVALID, "replay does not match its recording (shape, PSF, iso, maxit, h_bar request, "
                                        "lambda / rho, library options or the batch reducer (sharded or not) changed "
                                        "between record and replay)");
        if (use_masks && rho_bar)
            return fail(ADMM_E_INVALID, "recorded with ADMM_REC_MASKS (soft-threshold branches only / the fused isotropic "
                                        "trajectory): rho_bar cannot be formed from it; record without the flag to get rho_bar");
        g_rec.erase(it);
    } else {
        std::lock_guard<std::mutex> lk(g_rec_mu);
        if (phases == 1) g_rec[workspace] = tag;
        else g_rec.erase(workspace);
    }
    return launch_backward(phases, y, x_bar, y_bar, h_bar, lambda_bar, rho_bar, M, N, planes, h, kh, kw, sc, iso, maxit,
                           x_out, workspace, stream, red, plan, bl);
}

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
    L.two_pass = multi_two_pass(planes, flags);
    if (L.two_pass) {
        // the 2-pass kernels over every branch's planes (admm_launch.hip run_multi_2pass_*)
        const size_t ppb = planes / (size_t)nbr;
        const int T = bwd_line_T(kMultiM, kMultiN, iso);
        if (iso) {
            L.G = iso_group(ppb);
            L.ngb = iso_ngroups(ppb);
            L.nblk_a = L.ngb * (kMultiN / T);
            L.rows_b = L.nblk_a + kIsoAdjRBlocks;
        } else {
            L.rows_b = (int)ppb * (kMultiN / T);
        }
        L.pbs = (size_t)K * L.rows_b * 2;
        L.spec0 = take(planes * MN * 4);
        L.spec1 = take(planes * MN * 4);
        L.hln = take(planes * MN * 4);   // Y_h = F y per grid plane (H^T y in the spectral domain)
        if (iso) {
            L.fmap = take((size_t)nbr * MN * 4);
            L.qpart = take((size_t)nbr * L.ngb * MN * 4);
        }
        if (rec) {
            L.traj = take((size_t)(K > 1 ? K - 1 : 1) * planes * MN * 8);
            L.sbA = take(planes * MN * 8);
            L.sbB = take(planes * MN * 8);
            L.vsum = take(planes * MN * 4);
            L.part = take((size_t)nbr * L.pbs * 8);
            L.rt = take((size_t)nbr * 16);
            L.rtmp = take((size_t)kRedParts * 2 * 8);
            if (iso) {
                L.nrm = take((size_t)(K > 1 ? K - 1 : 1) * nbr * MN * 4);
                L.wbar = take(planes * MN * 4);
                L.rmap = take((size_t)nbr * MN * 4);
                L.Rpart = take((size_t)nbr * L.ngb * MN * 4);
            }
        } else {
            L.sA = take(planes * MN * 8);
            if (!iso) L.sbA = take(planes * MN * 8);   // the anisotropic s ping-pong's second buffer
        }
        L.total = off;
        return L;
    }
    L.F = take((size_t)nbr * multi_F_bytes());
    L.hln = take(admm::plane::hty_bytes(planes));   // lane-native H^T y at its skewed plane stride
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
    return launch_forward_multi(y, x_out, M, N, P, B, nbr, lambda, rho, maxit, flags, workspace, stream, planes, L);
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
    return launch_backward_multi(x_bar, y_bar, lambda_bar, rho_bar, M, N, P, B, nbr, maxit, x_out, workspace, stream,
                                 flags, planes, ppb, MN, L);
}

}  // namespace admm_capi

using namespace admm_capi;

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

int admm_clamp_backward_f32(const float* x, const float* dy, float* dx, size_t n, float lo, float hi, void* stream) {
    if (n == 0) return ADMM_OK;
    if (!x || !dy || !dx) return fail(ADMM_E_INVALID, "admm_clamp_backward_f32: NULL pointer");
    const size_t blocks = (n + 4 * 256 - 1) / (4 * 256);
    hipLaunchKernelGGL(admm::clamp_bwd_kernel, dim3((unsigned)(blocks < 65535 * 8 ? blocks : 65535 * 8)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), x, dy, dx, n, lo, hi);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(ADMM_E_HIP, "admm_clamp_backward_f32: %s", hipGetErrorString(e));
    return ADMM_OK;
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
