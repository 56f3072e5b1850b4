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
#include <mutex>
#include <string>
#include <vector>

#include "../../include/admm_deconv.h"
#include "admm_kernels.hip"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

bool is_pow2(int n) { return n > 0 && (n & (n - 1)) == 0; }

struct Layout {
    size_t twM, twN, C, G, hty, sA, sB, spec0, spec1, fmap, part, total;
};

size_t align_up(size_t v) { return (v + 255) & ~size_t(255); }

constexpr int kIsoGroup = 16;   // planes per ISO_A block (partial batch-norm sums)

Layout make_layout(int M, int N, size_t planes, bool psf, bool iso) {
    Layout L{};
    size_t off = 0;
    auto take = [&](size_t bytes) {
        size_t o = off;
        off = align_up(off + bytes);
        return o;
    };
    const size_t MN = (size_t)M * N;
    L.twM = take((size_t)M * 8);
    L.twN = take((size_t)N * 8);
    L.C = take((size_t)(M / 2 + 1) * N * 4);
    L.G = psf ? take((size_t)(M / 2 + 1) * N * 8) : 0;
    L.hty = psf ? take(planes * MN * 4) : 0;
    L.sA = take(planes * 2 * MN * 4);
    L.sB = take(planes * 2 * MN * 4);
    L.spec0 = take(planes * MN * 4);  // N lines x M/2 complex
    L.spec1 = take(planes * MN * 4);
    L.fmap = iso ? take(MN * 4) : 0;
    L.part = iso ? take(((planes + kIsoGroup - 1) / kIsoGroup) * MN * 4) : 0;
    L.total = off;
    return L;
}

// ---- tile-size policy ------------------------------------------------------------------------
// T = lines per line-kernel block (power of two dividing N); KB = slots per column-kernel block.
int line_T(int M, int N) {
    int pref = M <= 512 ? 8 : 4;
    if (const char* e = getenv("ADMM_LINE_T")) {
        int v = atoi(e);
        if (v == 2 || v == 4 || v == 8 || v == 16) pref = v < pref ? v : pref;
    }
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
int column_KB(int M, int N) {
    int KB = 256 / max_q(N);
    if (KB > M / 2) KB = M / 2;
    if (KB > 32) KB = 32;
    return KB;
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
    template <typename F>
    int run(int cls, F&& launch) {
        PendingEv p{cls, nullptr, nullptr};
        if (prof) {
            hipEventCreate(&p.a);
            hipEventCreate(&p.b);
            hipEventRecord(p.a, s);
        }
        launch();
        hipError_t e = hipGetLastError();
        if (prof) {
            hipEventRecord(p.b, s);
            ev.push_back(p);
        }
        if (e != hipSuccess) return fail(ADMM_E_HIP, "kernel launch (class %d) failed: %s", cls, hipGetErrorString(e));
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
                const float* so, float* sn, const float* hty, const float2* twM, int N, float tau, float rho,
                int sz) {
#define X(l, t)                                                                                          \
    if (L == l && T == t) {                                                                              \
        set_lds(line_kernel<l, t>, lds);                                                                 \
        line_kernel<l, t><<<g, kThreads, lds, s>>>(spec1, spec0, so, sn, hty, twM, N, tau, rho, sz);    \
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
                 const float* hty, float2* spec0, const float2* twM, int N, float rho) {
#define X(l, t)                                                                               \
    if (L == l && T == t) {                                                                   \
        set_lds(iso_b_kernel<l, t>, lds);                                                     \
        iso_b_kernel<l, t><<<g, kThreads, lds, s>>>(sn, fmap, hty, spec0, twM, N, rho);      \
        return 0;                                                                             \
    }
    ADMM_LT_CASES(X)
#undef X
    return -1;
}

int launch_column(int N, bool cplx, dim3 g, size_t lds, hipStream_t s, const float2* src, float2* dst,
                  const float* C, const float2* G, const float2* twN, int L, int KB, float cs) {
#define X(v)                                                                                 \
    if (N == v) {                                                                            \
        if (cplx) {                                                                          \
            set_lds(column_kernel<v, true>, lds);                                            \
            column_kernel<v, true><<<g, kThreads, lds, s>>>(src, dst, C, G, twN, L, KB, cs);  \
        } else {                                                                             \
            set_lds(column_kernel<v, false>, lds);                                           \
            column_kernel<v, false><<<g, kThreads, lds, s>>>(src, dst, C, G, twN, L, KB, cs); \
        }                                                                                    \
        return 0;                                                                            \
    }
    ADMM_N_CASES(X)
#undef X
    return -1;
}

int check_shape(int M, int N, int P, int B, int kh, int kw, int iso) {
    if (P < 1 || B < 1 || M < 1 || N < 1) return fail(ADMM_E_INVALID, "sizes must be positive (M=%d N=%d P=%d B=%d)", M, N, P, B);
    if (kh < 0 || kw < 0 || ((kh == 0) != (kw == 0)))
        return fail(ADMM_E_INVALID, "PSF size must be both zero (empty PSF) or both positive (kh=%d kw=%d)", kh, kw);
    if (!is_pow2(M) || !is_pow2(N) || M < 4 || M > 1024 || N < 2 || N > 1024)
        return fail(ADMM_E_UNSUPPORTED, "this build supports power-of-two 4<=M<=1024, 2<=N<=1024 (got M=%d N=%d)", M, N);
    if (kh > M || kw > N)
        return fail(ADMM_E_UNSUPPORTED, "PSF %dx%d larger than the image (kh<=M, kw<=N required, as pad_constant in ops.jl:25)", kh, kw);
    if (iso && (size_t)P * B > 65535)
        return fail(ADMM_E_UNSUPPORTED, "isotropic prox couples the batch: at most 65535 planes per call");
    return ADMM_OK;
}

}  // namespace

extern "C" {

int admm_abi_version(void) { return ADMM_ABI_VERSION; }

const char* admm_last_error(void) { return g_err.c_str(); }

int admm_tvd_workspace_bytes(int M, int N, int P, int B, int kh, int kw, int iso, size_t* out_bytes) {
    if (!out_bytes) return fail(ADMM_E_INVALID, "out_bytes is NULL");
    int rc = check_shape(M, N, P, B, kh, kw, iso);
    if (rc) return rc;
    *out_bytes = make_layout(M, N, (size_t)P * B, kh > 0, iso != 0).total;
    return ADMM_OK;
}

int admm_tvd_forward_f32(const float* y, float* x_out, int M, int N, int P, int B, const float* h, int kh, int kw,
                         float lambda, float rho, int iso, int maxit, void* workspace, size_t workspace_bytes,
                         void* stream) {
    if (h == nullptr) kh = kw = 0;
    int rc = check_shape(M, N, P, B, kh, kw, iso);
    if (rc) return rc;
    if (!y || !x_out) return fail(ADMM_E_INVALID, "y and x_out must be device pointers");
    if (maxit < 0) return fail(ADMM_E_INVALID, "maxit must be >= 0 (got %d)", maxit);
    if (!std::isfinite(lambda) || !std::isfinite(rho)) return fail(ADMM_E_INVALID, "lambda and rho must be finite");
    const size_t planes = (size_t)P * B;
    const Layout lay = make_layout(M, N, planes, kh > 0, iso != 0);
    if (!workspace || workspace_bytes < lay.total)
        return fail(ADMM_E_WORKSPACE, "workspace too small: need %zu bytes, got %zu", lay.total, workspace_bytes);
    if ((reinterpret_cast<uintptr_t>(workspace) & 255) != 0)
        return fail(ADMM_E_WORKSPACE, "workspace must be 256-byte aligned");
    if ((reinterpret_cast<uintptr_t>(y) & 15) || (reinterpret_cast<uintptr_t>(x_out) & 15))
        return fail(ADMM_E_INVALID, "y and x_out must be 16-byte aligned");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const size_t MN = (size_t)M * N;
    if (maxit == 0) {
        hipError_t e = hipMemsetAsync(x_out, 0, planes * MN * 4, s);
        if (e != hipSuccess) return fail(ADMM_E_HIP, "hipMemsetAsync: %s", hipGetErrorString(e));
        return ADMM_OK;
    }
    unsigned char* ws = static_cast<unsigned char*>(workspace);
    float2* twM = reinterpret_cast<float2*>(ws + lay.twM);
    float2* twN = reinterpret_cast<float2*>(ws + lay.twN);
    float* Ct = reinterpret_cast<float*>(ws + lay.C);
    float2* Gt = kh > 0 ? reinterpret_cast<float2*>(ws + lay.G) : nullptr;
    float* hty = kh > 0 ? reinterpret_cast<float*>(ws + lay.hty) : const_cast<float*>(y);
    float* sbuf[2] = {reinterpret_cast<float*>(ws + lay.sA), reinterpret_cast<float*>(ws + lay.sB)};
    float2* spec0 = reinterpret_cast<float2*>(ws + lay.spec0);
    float2* spec1 = reinterpret_cast<float2*>(ws + lay.spec1);
    const int L = M / 2;
    const float tau = lambda / rho;   // ops.jl:20

    Launcher ln{s, g_prof.on, {}};
    rc = ln.run(ADMM_K_SETUP, [&] {
        const size_t lds = (size_t)(M + N) * 16;
        const int nb = (int)(((size_t)(L + 1) * N + kThreads - 1) / kThreads);
        const int grid = nb < 1024 ? (nb < 1 ? 1 : nb) : 1024;
        hipLaunchKernelGGL(admm::setup_kernel, dim3(grid), dim3(kThreads), lds, s, twM, twN, Ct, Gt, h, kh, kw, M,
                           N, rho);
    });
    if (rc) return rc;

    const int T = line_T(M, N);
    const int KB = column_KB(M, N);
    const size_t llds = line_lds(M, T), flds = fwdinv_lds(M, T), clds = column_lds(N, KB);
    float* fmap = iso ? reinterpret_cast<float*>(ws + lay.fmap) : nullptr;
    float* part = iso ? reinterpret_cast<float*>(ws + lay.part) : nullptr;
    const int kMaxY = 65535;
    for (size_t p0 = 0; p0 < planes; p0 += kMaxY) {
        const int np = (int)((planes - p0) < (size_t)kMaxY ? (planes - p0) : (size_t)kMaxY);
        const float* yp = y + p0 * MN;
        float* htyp = hty + p0 * MN;
        float2* sp0 = spec0 + p0 * N * L;
        float2* sp1 = spec1 + p0 * N * L;
        float* sa = sbuf[0] + p0 * 2 * MN;
        float* sb = sbuf[1] + p0 * 2 * MN;
        float* xp = x_out + p0 * MN;
        const dim3 gl(N / T, np), gc(L / KB, np);
        // PREP: spectrum of y; with a PSF, H^T y = F^-1 conj(Sigma_c) F y (line, column, line)
        rc = ln.run(ADMM_K_PREP, [&] { launch_line_fwd(L, T, gl, flds, s, yp, sp0, twM, N); });
        if (rc) return rc;
        const float2* first = sp0;
        float cs1 = 1.0f;
        if (kh > 0) {
            rc = ln.run(ADMM_K_PREP, [&] { launch_column(N, true, gc, clds, s, sp0, sp1, Ct, Gt, twN, L, KB, 1.0f); });
            if (rc) return rc;
            rc = ln.run(ADMM_K_PREP, [&] { launch_line_inv(L, T, gl, flds, s, sp1, htyp, twM, N); });
            if (rc) return rc;
            first = sp1;          // = F_dim1(H^T y) / M
            cs1 = (float)M;
        }
        for (int it = 1; it <= maxit; ++it) {
            rc = ln.run(ADMM_K_COLUMN, [&] {
                launch_column(N, false, gc, clds, s, it == 1 ? first : sp0, sp1, Ct, Gt, twN, L, KB,
                              it == 1 ? cs1 : 1.0f);
            });
            if (rc) return rc;
            if (it < maxit && !iso) {
                float* so = (it & 1) ? sb : sa;   // iteration 1 reads nothing (s_zero)
                float* sn = (it & 1) ? sa : sb;
                rc = ln.run(ADMM_K_LINE, [&] {
                    launch_line(L, T, gl, llds, s, sp1, sp0, so, sn, htyp, twM, N, tau, rho, it == 1 ? 1 : 0);
                });
            } else if (it < maxit) {
                // isotropic: s is written in place (no halo reads of s in ISO_A)
                const int ng = (np + kIsoGroup - 1) / kIsoGroup;
                rc = ln.run(ADMM_K_LINE, [&] {
                    launch_iso_a(L, T, dim3(N / T, ng), iso_a_lds(M, T), s, sp1, sa, sa, fmap, part, twM, N, np,
                                 kIsoGroup, it == 1 ? 1 : 0);
                });
                if (rc) return rc;
                rc = ln.run(ADMM_K_NORM, [&] {
                    const int nb = (int)((MN + kThreads - 1) / kThreads);
                    hipLaunchKernelGGL(admm::iso_r_kernel, dim3(nb < 2048 ? nb : 2048), dim3(kThreads), 0, s, part,
                                       fmap, ng, MN, tau);
                });
                if (rc) return rc;
                rc = ln.run(ADMM_K_LINE, [&] {
                    launch_iso_b(L, T, gl, iso_b_lds(M, T), s, sa, fmap, htyp, sp0, twM, N, rho);
                });
            } else {
                rc = ln.run(ADMM_K_FINAL, [&] { launch_line_inv(L, T, gl, flds, s, sp1, xp, twM, N); });
            }
            if (rc) return rc;
        }
    }
    return ln.finish();
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

}  // extern "C"
