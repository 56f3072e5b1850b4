/*
 * admm_deconv.h -- C ABI of the MI355X-native ADMM TV-deconvolution solve.
 *
 * This is the drop-in boundary for the reference's hot path
 *   tvd_fft(y, λ, ρ, h, isotropic=false, maxit=100)          /root/reference/src/ops/ops.jl:181-188
 * whose two bodies are tvd_fft_cpu (ops.jl:17-96) and tvd_fft_gpu (ops.jl:99-178).  The
 * reference reaches it from the Flux layer forward `(d::Admm)(x)` (src/layers/deconv_admm.jl:215-225),
 * which clamps λ, ρ and the PSF first; callers of this ABI pass the already-clamped fp32 values.
 * The Julia `ccall` binding a maintainer would add, and the Python ctypes binding this repo uses,
 * are shown in INTEGRATION.md.
 *
 * Conventions
 *  - Every array pointer is a DEVICE pointer owned by the caller.  Layout is the reference's
 *    column-major Julia array (M,N,P,B) == C `float[B][P][N][M]` (dim1 = M contiguous).
 *    The PSF h is Julia (kh,kw,1,1) == C `float[kw][kh]`; kh == kw == 0 (or h == NULL) is the
 *    reference's empty PSF (`isempty(h)` -> H = identity, ops.jl:22-23,67-69).
 *  - The library allocates nothing in the solve: the caller supplies a device workspace of at
 *    least admm_tvd_workspace_bytes() bytes (256-byte aligned).  Work is enqueued on `stream`
 *    (a hipStream_t, NULL = default stream) and is asynchronous, like CUDA.jl's task-local stream.
 *    `y` is never modified; the result goes to `x_out` (the reference returns a new array).
 *  - Return value: 0 on success, a negative ADMM_E* code otherwise; admm_last_error() gives a
 *    thread-local message for the last failing call.
 *  - Supported shapes: any 2 <= M, N <= 4096 with kh <= M, kw <= N (the reference accepts any
 *    M x N >= 2 x 2 through FFTW/CUFFT).  Powers of two with 4 <= M <= 1024, 2 <= N <= 1024 run
 *    the tuned kernels; every other shape runs a runtime-length mixed-radix path (forward and
 *    adjoint).
 */
#ifndef ADMM_DECONV_H
#define ADMM_DECONV_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ADMM_ABI_VERSION 3

enum {
    ADMM_OK = 0,
    ADMM_E_INVALID = -1,      /* bad argument (null pointer, negative size, non-finite λ/ρ) */
    ADMM_E_UNSUPPORTED = -2,  /* shape/option outside this build's support matrix           */
    ADMM_E_WORKSPACE = -3,    /* workspace too small or misaligned                          */
    ADMM_E_HIP = -4,          /* a HIP runtime call failed (message has hipGetErrorString)   */
    ADMM_E_REDUCER = -5       /* the caller's batch reducer (admm_batch_reducer) failed       */
};

/* Kernel classes, for the optional per-kernel profiler (admm_profile_*). */
enum {
    ADMM_K_SETUP = 0,   /* twiddles + C spectrum (ops.jl:22-37)                                 */
    ADMM_K_PREP = 1,    /* H^T y (ops.jl:71-81) + first line rFFT                                */
    ADMM_K_COLUMN = 2,  /* column pass: FFT along dim2, x C, IFFT along dim2 (ops.jl:86 part)    */
    ADMM_K_LINE = 3,    /* line pass: irFFT dim1 -> D -> prox -> dual -> D^T -> +H^T y -> rFFT   */
    ADMM_K_FINAL = 4,   /* last irFFT along dim1, writes x                                       */
    ADMM_K_NORM = 5,    /* isotropic only: pixelnorm over the batch (ops.jl:6)                   */
    ADMM_K_PLANE = 6,   /* fused per-plane solve, all K iterations (256 x 256, anisotropic)      */
    ADMM_K_ADJ = 7,     /* adjoint reverse-step kernels (line_adj, iso_adj_a / iso_adj_b, fused)  */
    ADMM_K_COUNT = 8
};

/* ABI version of the loaded library (== ADMM_ABI_VERSION it was built with). */
int admm_abi_version(void);

/* Thread-local message describing the most recent failure ("" if none). */
const char* admm_last_error(void);

/* Workspace size for one tvd_fft call of this shape.  Replaces the allocations
 * tvd_fft_gpu makes internally (ops.jl:104-131, fresh temporaries every iteration). */
int admm_tvd_workspace_bytes(int M, int N, int P, int B, int kh, int kw, int iso,
                             size_t* out_bytes);

/* The solve.  Replaces tvd_fft(y, λ, ρ, h, isotropic, maxit) (ops.jl:181-188) for device
 * arrays: returns x after `maxit` ADMM iterations of
 *   x = irfft(C .* rfft(H^T y + ρ D^T(z-u))),  z = prox(Dx+u, λ/ρ),  u = u + Dx - z
 * with prox = ST (iso == 0, ops.jl:9) or BT (iso == 1, ops.jl:10; couples the whole batch).
 * maxit == 0 returns zeros (the reference's initial x, ops.jl:46).
 * Batch size: iso == 1 takes at most 65535 planes (P*B) per call.  iso == 0 takes any number; above
 * 65,280 planes the library solves consecutive chunks of 65,280 planes through one chunk-sized
 * workspace (admm_tvd_workspace_bytes sizes it).  The adjoint entry points below take at most 65535
 * planes per call. */
int admm_tvd_forward_f32(const float* y, float* x_out, int M, int N, int P, int B,
                         const float* h, int kh, int kw, float lambda, float rho, int iso,
                         int maxit, void* workspace, size_t workspace_bytes, void* stream);

/* Adjoint of admm_tvd_forward_f32 (the Zygote reverse pass through the K unrolled iterations that
 * the reference's training uses, src/train.jl:51 with src/ops/ops.jl:84-92; BASELINE config c5).
 * Recomputes the forward (writing x to x_out) while recording one state tensor per iteration, then
 * runs the reverse sweep.  Given x_bar = dL/dx it writes
 *   y_bar (device, shape of y; NULL = not needed, cheaper: with h_bar also NULL the reverse sweep
 *          keeps no running sum of vbar, 8 B/px less HBM traffic per reverse step)
 *   h_bar (device, kw*kh floats; NULL = not needed, cheaper)
 *   lambda_bar, rho_bar (device, 1 float each; NULL = not needed)
 * Both proxes: with iso != 0 the trajectory also keeps the per-pixel batch norm of every s_k and
 * each reverse step reduces R = sum over planes of s (2 w_bar - s_bar) across the batch.
 * Deterministic (fixed reduction order). */
int admm_tvd_backward_workspace_bytes(int M, int N, int P, int B, int kh, int kw, int iso, int maxit,
                                      int want_hbar, size_t* out_bytes);
int admm_tvd_backward_f32(const float* y, const float* x_bar, float* y_bar, float* h_bar,
                          float* lambda_bar, float* rho_bar, int M, int N, int P, int B,
                          const float* h, int kh, int kw, float lambda, float rho, int iso, int maxit,
                          float* x_out, void* workspace, size_t workspace_bytes, void* stream);

/* Sharded batch for the isotropic prox.  BT's pixelnorm sums s^2 over EVERY plane of
 * the batch (ops.jl:6), so when the batch is split across processes (one per GPU) each iteration
 * needs the cross-shard sum of one M x N fp32 map.  The library calls
 *     fn(buf, count, stream, user)
 * with `buf` a device pointer into the workspace holding this shard's `count` = M*N partial sums;
 * fn must replace them, in place, by the element-wise sum over all shards, ordered after the work
 * already enqueued on `stream` and before work enqueued on `stream` after it returns (an
 * ncclAllReduce(sum) on `stream`, or torch.distributed.all_reduce on the stream's torch twin).
 * Every shard must make the same sequence of calls.  fn returns 0 on success; a non-zero return
 * aborts the solve with ADMM_E_REDUCER.  The forward calls it K-1 times (pixelnorm of s_1..s_{K-1});
 * the backward K-1 times more (the batch map R of each reverse step).  Backward outputs are this
 * shard's: y_bar for its planes, and its CONTRIBUTION to h_bar / lambda_bar / rho_bar (sum them over
 * shards, as data-parallel training all-reduces every parameter gradient).
 * With iso == 0 the reducer is ignored (planes are independent).  reducer == NULL (or fn == NULL)
 * is the unsharded call, identical to admm_tvd_forward_f32 / admm_tvd_backward_f32.  A sharded
 * isotropic call ignores the plane-count rule (ADMM_OPT_MIN_PLANES): every shard takes the per-plane
 * kernels whatever its own size, so that all shards hand the reducer their maps in one layout.  A recording
 * remembers whether it was made with a reducer: its replay must pass one too (or none), else ADMM_E_INVALID. */
typedef int (*admm_reduce_fn)(float* buf, size_t count, void* stream, void* user);
typedef struct {
    admm_reduce_fn fn;
    void* user;
} admm_batch_reducer;

int admm_tvd_forward_sharded_f32(const float* y, float* x_out, int M, int N, int P, int B,
                                 const float* h, int kh, int kw, float lambda, float rho, int iso,
                                 int maxit, void* workspace, size_t workspace_bytes, void* stream,
                                 const admm_batch_reducer* reducer);
int admm_tvd_backward_sharded_f32(const float* y, const float* x_bar, float* y_bar, float* h_bar,
                                  float* lambda_bar, float* rho_bar, int M, int N, int P, int B,
                                  const float* h, int kh, int kw, float lambda, float rho, int iso,
                                  int maxit, float* x_out, void* workspace, size_t workspace_bytes,
                                  void* stream, const admm_batch_reducer* reducer);

/* Split adjoint for a training step: the forward records its trajectory into `workspace` (sized by
 * admm_tvd_backward_workspace_bytes with the same arguments and want_hbar), the backward later runs
 * only the reverse sweep from it -- the forward is not recomputed.  Between the two calls the
 * workspace must not be touched and x_out must still hold the recorded forward's output; y, h,
 * lambda, rho, iso, maxit and the library options (admm_set_option) must be the same.  h_bar must be
 * non-NULL in the backward iff want_hbar was set in the forward.  With a reducer (iso, sharded
 * batch) both calls must get one.  admm_tvd_backward_f32 is exactly the two calls back to back.
 * The library remembers, per workspace, the arguments and options a recording was made with: a replay
 * that differs (or a workspace that holds no recording -- a plain forward on it overwrites one)
 * fails with ADMM_E_INVALID rather than reading a trajectory of another layout.  A recording is
 * consumed by its replay. */
/* `want_hbar` of the record entry points (and of admm_tvd_backward_workspace_bytes) is a flag word:
 *   ADMM_REC_HBAR  (1): also record what h_bar needs (the replay must then be given h_bar);
 *   ADMM_REC_MASKS (2): the replay will not be asked for rho_bar -- record only the soft-threshold
 *       branch of every trajectory element (1[|s_k| > tau] and sign(s_k), 1 byte per pixel pair and
 *       iteration) instead of s_k itself: 16x less trajectory memory and, in the fused
 *       256 x 256 anisotropic reverse sweep, 8 of its 24 B/px per step gone.  lambda_bar, y_bar and h_bar
 *       are bitwise those of a full recording; a replay with rho_bar != NULL fails with ADMM_E_INVALID.
 *       Honoured by the fused anisotropic trajectory (256 x 256, no h_bar); isotropic at 256 x 256 (no
 *       h_bar) it selects the fused isotropic sweep instead (plane_iso.hip: s_k and |s_k| kept in the
 *       kernels' lane-native layout, no rho_bar either), also for a sharded batch: the reducer then sums
 *       the R map of every reverse step over the shards before s_bar is formed, while lambda_bar is this
 *       shard's partial (tau_bar from the shard's own R), so the caller sums lambda_bar over the shards as
 *       it does for the 2-pass sweep; elsewhere the full trajectory is recorded and rho_bar stays
 *       available. */
enum { ADMM_REC_HBAR = 1, ADMM_REC_MASKS = 2 };

int admm_tvd_forward_record_f32(const float* y, float* x_out, int M, int N, int P, int B,
                                const float* h, int kh, int kw, float lambda, float rho, int iso,
                                int maxit, int want_hbar, void* workspace, size_t workspace_bytes,
                                void* stream, const admm_batch_reducer* reducer);
int admm_tvd_backward_recorded_f32(const float* y, const float* x_bar, float* y_bar, float* h_bar,
                                   float* lambda_bar, float* rho_bar, int M, int N, int P, int B,
                                   const float* h, int kh, int kw, float lambda, float rho, int iso,
                                   int maxit, const float* x_out, void* workspace,
                                   size_t workspace_bytes, void* stream,
                                   const admm_batch_reducer* reducer);

/* Device-resident λ and ρ.  The reference operator takes them as 1-element device arrays,
 * tvd_fft(y, λ::CGPUArray, ρ::CGPUArray, h, ...) (ops.jl:99,181), and the layer clamps them on the
 * device (deconv_admm.jl:216-217).  These entry points take `lambda` and `rho` as DEVICE pointers to
 * one fp32 each, read in-kernel (τ = λ/ρ is formed on the device), so a training step never reads
 * them back to the host.  Otherwise identical to the host-scalar entry points above; `reducer` may be
 * NULL (unsharded).  The values must be finite and ρ > 0 (not checked: checking would need a host
 * read); the reference has no guard either. */
int admm_tvd_forward_dev_f32(const float* y, float* x_out, int M, int N, int P, int B,
                             const float* h, int kh, int kw, const float* lambda, const float* rho,
                             int iso, int maxit, void* workspace, size_t workspace_bytes, void* stream,
                             const admm_batch_reducer* reducer);
int admm_tvd_backward_dev_f32(const float* y, const float* x_bar, float* y_bar, float* h_bar,
                              float* lambda_bar, float* rho_bar, int M, int N, int P, int B,
                              const float* h, int kh, int kw, const float* lambda, const float* rho,
                              int iso, int maxit, float* x_out, void* workspace,
                              size_t workspace_bytes, void* stream, const admm_batch_reducer* reducer);
int admm_tvd_forward_record_dev_f32(const float* y, float* x_out, int M, int N, int P, int B,
                                    const float* h, int kh, int kw, const float* lambda,
                                    const float* rho, int iso, int maxit, int want_hbar,
                                    void* workspace, size_t workspace_bytes, void* stream,
                                    const admm_batch_reducer* reducer);
int admm_tvd_backward_recorded_dev_f32(const float* y, const float* x_bar, float* y_bar,
                                       float* h_bar, float* lambda_bar, float* rho_bar, int M, int N,
                                       int P, int B, const float* h, int kh, int kw,
                                       const float* lambda, const float* rho, int iso, int maxit,
                                       const float* x_out, void* workspace, size_t workspace_bytes,
                                       void* stream, const admm_batch_reducer* reducer);

/* Several solves of ONE shared input in one launch: the branches of a Flux
 * `Parallel(chcat, b_1, ..., b_nbranch)` whose branches are ADMM layers without a PSF (the denoiser,
 * src/nets/net_build.jl:113-125: five ADMMDeconvF2((), 50, ρ_i, relu1)).  Branch i solves every plane
 * of y with its own λ_i, ρ_i (device pointers: lambda[i], rho[i] -- host arrays of `nbranch` device
 * pointers) and writes the chcat layout: x_out is Julia (M, N, nbranch*P, B) == C
 * `float[B][nbranch*P][N][M]`, branch i's channels at i*P .. i*P+P-1 -- the output of
 * `Parallel(chcat, ...)` itself, before the layers' bias / σ.  All nbranch*P*B planes run in one grid --
 * of the fused kernels, or, below the plane-count rule (ADMM_OPT_MIN_PLANES at its default: fewer than 96
 * planes in all anisotropic / 112 isotropic), of the 2-pass kernels, which spread every plane over many
 * workgroups (the training batch of 2: 30 planes) -- so no CU idles between branches.  256 x 256, no PSF,
 * at most 65,280 planes in total (nbranch*P*B); the same results, bitwise, as nbranch separate solves
 * through the same kernels.  The workspace size follows the rule (admm_tvd_multi_workspace_bytes).
 * flags: ADMM_MULTI_RECORD (1) records the trajectory for admm_tvd_backward_multi_recorded_dev_f32
 *        (the workspace then holds it until the replay); | ADMM_REC_MASKS (2) as above (no rho_bar);
 *        | ADMM_MULTI_ISO (4): isotropic prox (use_iso) -- the split-iteration kernels of plane_iso.hip,
 *        each branch's batch norm over its own planes; its recording never gives rho_bar.
 * The backward writes lambda_bar[i] (and rho_bar[i]; device arrays of nbranch floats, NULL = not
 * needed; rho_bar must be NULL with ADMM_REC_MASKS) and y_bar = the sum over branches of each branch's
 * input gradient (NULL = not needed, cheaper), from x_bar in the chcat layout of x_out.  x_out must
 * still hold the recorded output. */
enum { ADMM_MULTI_RECORD = 1, ADMM_MULTI_ISO = 4 };
int admm_tvd_multi_workspace_bytes(int M, int N, int P, int B, int nbranch, int maxit, int flags,
                                   size_t* out_bytes);
int admm_tvd_forward_multi_dev_f32(const float* y, float* x_out, int M, int N, int P, int B, int nbranch,
                                   const float* const* lambda, const float* const* rho, int maxit, int flags,
                                   void* workspace, size_t workspace_bytes, void* stream);
int admm_tvd_backward_multi_recorded_dev_f32(const float* x_bar, float* y_bar, float* lambda_bar,
                                             float* rho_bar, int M, int N, int P, int B, int nbranch,
                                             int maxit, const float* x_out, void* workspace,
                                             size_t workspace_bytes, void* stream);

/* Library options: process-global switches read at each call.  The defaults are the tuned choices;
 * the others exist for tests (fused vs 2-pass paths) and tuning experiments.  Not read from the
 * environment.  A recording remembers the options it was made with (see above). */
enum {
    ADMM_OPT_FUSED = 0,          /* 1 (default): fused per-plane kernel at 256x256 anisotropic; 0: 2-pass */
    ADMM_OPT_FUSED_ADJ = 1,      /* 1 (default): fused reverse sweep on a fused trajectory; 0: 2-pass    */
    ADMM_OPT_LINE_T = 2,         /* 0 (default): tile policy; 2/4/8/16: cap on lines per line block      */
    ADMM_OPT_COL_THREADS = 3,    /* 0 (default): policy; 256, 512 or 1024 threads per column block       */
    ADMM_OPT_GEN_TM = 4,         /* 0 (default 2048): runtime-length line block points, 256..8192        */
    ADMM_OPT_GEN_KN = 5,         /* 0 (default 1024): runtime-length column block points, 256..8192      */
    ADMM_OPT_PLANE_STAGGER = 6,  /* retired (round 6): the start-delay experiment left the kernels; the value
                                    is still stored and read back, and changes nothing                     */
    ADMM_OPT_SMOOTH = 7,         /* 1 (default): compile-time-plan kernels for the listed non-power-of-two
                                    lengths (admm_smooth.hip); 0: runtime plans for every such shape;
                                    2 / 3: compiled, column plans forced increasing / decreasing (sweeps)  */
    ADMM_OPT_RESIDENT = 8,       /* 1 (default): one workgroup per plane runs all K iterations for the smooth
                                    non-power-of-two shapes admm_resident.hip compiled and measured faster
                                    (anisotropic, no h_bar trajectory); 2: every compiled shape; 0: the
                                    2-pass smooth kernels                                                     */
    ADMM_OPT_MIN_PLANES = 9,     /* -1 (default): the one-workgroup-per-plane paths (fused, fused_iso, resident,
                                    resident_iso) are taken only from the measured plane counts where they beat
                                    the multi-workgroup 2-pass kernels (admm_capi.hip kMinPlanes; a smaller batch
                                    runs the 2-pass kernels, so a plane's result can differ by fp32 rounding
                                    between batch sizes); 0: those paths at every batch size (results independent
                                    of the batch size, as for anisotropic solves before); n > 0: from n planes  */
    ADMM_OPT_MALL_STREAMS = 10,  /* 4 (default): an anisotropic 2-pass forward (power-of-two, smooth or runtime
                                    lengths) whose per-iteration working set (28 B/px: spectrum in / out, s in /
                                    out, Y_h) is over twice the 256 MiB Infinity Cache runs as plane chunks of
                                    ~224 MiB / n (at least 4 planes, else the whole batch), n chunks at a time
                                    on the caller's stream and n - 1 library streams (each chunk all K
                                    iterations, its set cache-resident; bitwise the whole-batch solve;
                                    workspace n chunks; admm_query_forward_schedule);
                                    0 or 1: the whole batch on the caller's stream                           */
    ADMM_OPT_COUNT = 11
};
int admm_set_option(int option, int value);
int admm_get_option(int option, int* value);

/* Which kernels a call runs (one decision table in admm_capi.hip, plan_paths; measurement and tests only).
 * mode: ADMM_MODE_FORWARD (admm_tvd_forward_*), ADMM_MODE_RECORD (admm_tvd_forward_record_*; flags =
 * its ADMM_REC_* word; its replay runs the sweep returned here), ADMM_MODE_BACKWARD (admm_tvd_backward_*;
 * want_hbar / want_rho = h_bar / rho_bar non-NULL).  kh = 0: no PSF.  planes = P * B of the call (0: not known,
 * no plane-count rule, see ADMM_OPT_MIN_PLANES; a sharded call -- a batch reducer given -- is planned as planes = 0,
 * so query it with 0).  *fwd_path = the forward's ADMM_PATH_*,
 * *bwd_path = the reverse sweep's ADMM_PATH_SWEEP_* (0 for a plain forward).  The current library options
 * (admm_set_option) are taken into account; no GPU is touched.  The multi-branch entry points are not
 * covered (one grid of the fused kernels, or ADMM_E_UNSUPPORTED). */
enum { ADMM_MODE_FORWARD = 0, ADMM_MODE_RECORD = 1, ADMM_MODE_BACKWARD = 2 };
enum {
    ADMM_PATH_FUSED = 1,              /* 256 x 256 anisotropic: plane256_kernel, one launch per solve         */
    ADMM_PATH_FUSED_ISO = 2,          /* 256 x 256 isotropic: plane256_iso_kernel + iso_norm_kernel / iter    */
    ADMM_PATH_2PASS = 3,              /* other power-of-two shapes: column_kernel + line_kernel per iteration */
    ADMM_PATH_2PASS_ISO = 4,          /* power-of-two isotropic: column + iso_a / iso_r / iso_b               */
    ADMM_PATH_RESIDENT = 5,           /* smooth squares <= 256: resident_kernel, one launch per solve         */
    ADMM_PATH_SMOOTH = 6,             /* compile-time plans for a smooth length (admm_smooth.hip)             */
    ADMM_PATH_RUNTIME = 7,            /* runtime plans for any length (admm_generic.hip)                      */
    ADMM_PATH_SWEEP_FUSED = 8,        /* plane256_adj_kernel, one launch per sweep                            */
    ADMM_PATH_SWEEP_FUSED_ISO = 9,    /* plane256_isoadj_kernel + iso_radj_kernel per step                   */
    ADMM_PATH_SWEEP_2PASS = 10,       /* line_adj + column per step                                          */
    ADMM_PATH_SWEEP_2PASS_ISO = 11,   /* iso_adj_a / _r / _b + column per step                                */
    ADMM_PATH_SWEEP_RUNTIME = 12,     /* admm_generic_bwd.hip                                                 */
    ADMM_PATH_SWEEP_RUNTIME_ISO = 13,
    ADMM_PATH_RESIDENT_ISO = 14       /* sides <= 256 isotropic: resident_iso_kernel + norm kernel per iteration */
};
int admm_query_paths(int M, int N, int iso, int kh, long long planes, int mode, int flags, int want_hbar, int want_rho,
                     int* fwd_path, int* bwd_path);
const char* admm_path_name(int path);
/* The forward's plane schedule for a call of `planes` = P*B planes (host only, ADMM_OPT_MALL_STREAMS): the planes
 * per launch (*chunk_planes) and the number of streams the chunks run on (*streams; 1 = the caller's stream only,
 * chunks back to back).  For tests and tooling, e.g. to price one launch's bytes.  ADMM_E_INVALID as
 * admm_query_paths. */
int admm_query_forward_schedule(int M, int N, int iso, int kh, long long planes, long long* chunk_planes,
                                int* streams);

/* The gradient of the layers' clamp activations (sigma = relu1 = min.(relu.(x), 1), src/nets/net_build.jl:8, and
 * relu6): dx[i] = (lo <= x[i] <= hi) ? dy[i] : 0 over n floats in one pass (autograd's form of the clamp is three
 * kernels).  x, dy, dx device pointers (dx may be dy); ADMM_E_INVALID for NULL pointers when n > 0. */
int admm_clamp_backward_f32(const float* x, const float* dy, float* dx, size_t n, float lo, float hi, void* stream);

/* Output transport of the batch-sharded solve (BASELINE c3; the reference gathers nothing -- its batch
 * lives on one device, ops.jl:168-173): an asynchronous copy of `bytes` from src to dst on `stream`, both
 * device pointers, dst possibly memory of another GPU opened through a HIP IPC handle.  A plain
 * hipMemcpyAsync on the caller's stream: the runtime gives device-to-device copies between GPUs of at
 * least ROC_P2P_SDMA_SIZE (1 MiB by default) to an SDMA engine, so the transfer holds no CU and touches
 * no HIP stream of the peer device.  ADMM_E_INVALID for NULL pointers, ADMM_E_HIP if the runtime refuses. */
int admm_copy_async(void* dst, const void* src, size_t bytes, void* stream);

/* The receive buffer of that transport, shared once per run through a HIP IPC handle (no counterpart in
 * the reference).  admm_ipc_get_handle: the ADMM_IPC_HANDLE_BYTES-byte handle of the device allocation
 * that holds dev_ptr (a caching allocator's block may sit inside a larger allocation) and dev_ptr's byte
 * offset in it.  admm_ipc_open: maps a peer process's handle into THIS process on `device` (the caller's
 * own GPU; the current device is restored) with lazy peer access, *dev_ptr_out = the allocation's base
 * (add the offset).  No context, stream or queue is created on the peer's GPU.  admm_ipc_close unmaps it.
 * ADMM_E_INVALID for NULL pointers, ADMM_E_HIP if the runtime refuses. */
#define ADMM_IPC_HANDLE_BYTES 64
int admm_ipc_get_handle(const void* dev_ptr, void* handle_out, size_t* offset_out);
int admm_ipc_open(const void* handle, int device, void** dev_ptr_out);
int admm_ipc_close(void* dev_ptr, int device);

/* Optional per-kernel timing (measurement only; off by default).  When enabled, each launch
 * inside admm_tvd_forward_f32 is bracketed by hipEvents on `stream` and the call synchronises
 * the stream before returning.  admm_profile_get returns the accumulated device time (ms) and
 * launch count of one ADMM_K_* class since the last reset. */
int admm_profile_enable(int on);
int admm_profile_reset(void);
int admm_profile_get(int kernel_class, double* total_ms, long long* launches);

#ifdef __cplusplus
}
#endif

#endif /* ADMM_DECONV_H */
