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
    size_t twM, twN, C, hty, sA, sB, spec0, spec1, total;
};

size_t align_up(size_t v) { return (v + 255) & ~size_t(255); }

Layout make_layout(int M, int N, size_t planes, bool psf) {
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
    L.hty = psf ? take(planes * MN * 4) : 0;
    L.sA = take(planes * 2 * MN * 4);
    L.sB = take(planes * 2 * MN * 4);
    L.spec0 = take(planes * MN * 4);  // N lines x M/2 complex
    L.spec1 = take(planes * MN * 4);
    L.total = off;
    return L;
}

// ---- tile-size policy ------------------------------------------------------------------------
constexpr size_t kLdsBudget = 96 * 1024;

int line_T(int M, int N) {  // largest power-of-two T <= 16 dividing N whose LDS fits
    int T = N < 16 ? N : 16;
    while (T > 1) {
        const size_t L = M / 2;
        const size_t bytes = (size_t)M * 8 + 2 * (size_t)(T + 2) * L * 8 + (size_t)T * M * 4;
        if (bytes <= kLdsBudget) break;
        T >>= 1;
    }
    return T;
}
size_t line_lds(int M, int T) {
    const size_t L = M / 2;
    return (size_t)M * 8 + 2 * (size_t)(T + 2) * L * 8 + (size_t)T * M * 4;
}
size_t final_lds(int M, int T) { return (size_t)M * 8 + 2 * (size_t)T * (M / 2) * 8; }
size_t prep_lds(int M, int T, int kh, int kw) {
    size_t b = final_lds(M, T);
    if (kh > 0) b += (size_t)((kh * kw + 3) & ~3) * 4 + (size_t)(T + kw - 1) * M * 4;
    return b;
}
int prep_T(int M, int N, int kh, int kw) {
    int T = N < 16 ? N : 16;
    while (T > 1 && prep_lds(M, T, kh, kw) > kLdsBudget) T >>= 1;
    return T;
}
int column_KB(int M, int N) {
    const int L = M / 2;
    int KB = 16;
    while (KB > 1 && (size_t)KB * N > 4096) KB >>= 1;
    if (KB > L) KB = L;
    return KB;
}
size_t column_lds(int N, int KB) { return (size_t)N * 8 + 2 * (size_t)KB * (N + 1) * 8; }

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

#define ADMM_L_CASES(X) X(2) X(4) X(8) X(16) X(32) X(64) X(128) X(256) X(512)
#define ADMM_N_CASES(X) X(2) X(4) X(8) X(16) X(32) X(64) X(128) X(256) X(512) X(1024)

using namespace admm;

int launch_prep(int L, dim3 g, size_t lds, hipStream_t s, const float* y, float* hty, float2* spec0,
                const float* h, int kh, int kw, const float2* twM, int N, int T) {
    switch (L) {
#define X(v)                                                                                  \
    case v:                                                                                   \
        hipFuncSetAttribute((const void*)prep_kernel<v>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
        prep_kernel<v><<<g, kThreads, lds, s>>>(y, hty, spec0, h, kh, kw, twM, N, T);          \
        return 0;
        ADMM_L_CASES(X)
#undef X
    }
    return -1;
}

int launch_line(int L, dim3 g, size_t lds, hipStream_t s, const float2* spec1, float2* spec0, const float* so,
                float* sn, const float* hty, const float2* twM, int N, int T, float tau, float rho, int sz) {
    switch (L) {
#define X(v)                                                                                  \
    case v:                                                                                   \
        hipFuncSetAttribute((const void*)line_kernel<v>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
        line_kernel<v><<<g, kThreads, lds, s>>>(spec1, spec0, so, sn, hty, twM, N, T, tau, rho, sz); \
        return 0;
        ADMM_L_CASES(X)
#undef X
    }
    return -1;
}

int launch_final(int L, dim3 g, size_t lds, hipStream_t s, const float2* spec1, float* x, const float2* twM, int N,
                 int T) {
    switch (L) {
#define X(v)                                                                                  \
    case v:                                                                                   \
        hipFuncSetAttribute((const void*)final_kernel<v>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
        final_kernel<v><<<g, kThreads, lds, s>>>(spec1, x, twM, N, T);                        \
        return 0;
        ADMM_L_CASES(X)
#undef X
    }
    return -1;
}

int launch_column(int N, dim3 g, size_t lds, hipStream_t s, const float2* spec0, float2* spec1, const float* C,
                  const float2* twN, int L, int KB) {
    switch (N) {
#define X(v)                                                                                  \
    case v:                                                                                   \
        hipFuncSetAttribute((const void*)column_kernel<v>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
        column_kernel<v><<<g, kThreads, lds, s>>>(spec0, spec1, C, twN, L, KB);               \
        return 0;
        ADMM_N_CASES(X)
#undef X
    }
    return -1;
}

int check_shape(int M, int N, int P, int B, int kh, int kw, int iso) {
    if (P < 1 || B < 1 || M < 1 || N < 1) return fail(ADMM_E_INVALID, "sizes must be positive (M=%d N=%d P=%d B=%d)", M, N, P, B);
    if (kh < 0 || kw < 0 || ((kh == 0) != (kw == 0)))
        return fail(ADMM_E_INVALID, "PSF size must be both zero (empty PSF) or both positive (kh=%d kw=%d)", kh, kw);
    if (!is_pow2(M) || !is_pow2(N) || M < 4 || M > 1024 || N < 2 || N > 1024)
        return fail(ADMM_E_UNSUPPORTED, "this build supports power-of-two 4<=M<=1024, 2<=N<=1024 (got M=%d N=%d)", M, N);
    if (kh > M || kw > N || kh * kw > 4096)
        return fail(ADMM_E_UNSUPPORTED, "PSF %dx%d larger than supported (kh<=M, kw<=N, kh*kw<=4096)", kh, kw);
    if (iso) return fail(ADMM_E_UNSUPPORTED, "isotropic (BT) prox is not in this build yet");
    if (prep_lds(M, prep_T(M, N, kh, kw), kh, kw) > 160 * 1024) return fail(ADMM_E_UNSUPPORTED, "PSF tile exceeds LDS");
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
    *out_bytes = make_layout(M, N, (size_t)P * B, kh > 0).total;
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
    const Layout lay = make_layout(M, N, planes, kh > 0);
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
    float* Cm = reinterpret_cast<float*>(ws + lay.C);
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
        hipLaunchKernelGGL(admm::setup_kernel, dim3(grid), dim3(kThreads), lds, s, twM, twN, Cm, h, kh, kw, M, N, rho);
    });
    if (rc) return rc;

    const int Tp = prep_T(M, N, kh, kw), Tl = line_T(M, N), Tf = line_T(M, N);
    const int KB = column_KB(M, N);
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
        rc = ln.run(ADMM_K_PREP, [&] {
            launch_prep(L, dim3(N / Tp, np), prep_lds(M, Tp, kh, kw), s, yp, kh > 0 ? htyp : nullptr, sp0, h, kh, kw,
                        twM, N, Tp);
        });
        if (rc) return rc;
        for (int it = 1; it <= maxit; ++it) {
            rc = ln.run(ADMM_K_COLUMN, [&] {
                launch_column(N, dim3(L / KB, np), column_lds(N, KB), s, sp0, sp1, Cm, twN, L, KB);
            });
            if (rc) return rc;
            if (it < maxit) {
                float* so = (it & 1) ? sb : sa;   // iteration 1 reads nothing (s_zero)
                float* sn = (it & 1) ? sa : sb;
                rc = ln.run(ADMM_K_LINE, [&] {
                    launch_line(L, dim3(N / Tl, np), line_lds(M, Tl), s, sp1, sp0, so, sn, htyp, twM, N, Tl, tau, rho,
                                it == 1 ? 1 : 0);
                });
            } else {
                rc = ln.run(ADMM_K_FINAL, [&] {
                    launch_final(L, dim3(N / Tf, np), final_lds(M, Tf), s, sp1, xp, twM, N, Tf);
                });
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
