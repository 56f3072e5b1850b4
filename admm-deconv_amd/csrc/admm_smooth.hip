// admm_smooth.hip -- the runtime-length path's per-iteration kernels with compile-time plans.
//
// The reference solves any M x N (ops.jl:86 / :168 through FFTW / CUFFT plans of the image size).
// admm_generic.hip covers every shape with runtime plans; its per-iteration kernels spend most of their
// time on runtime-radix loops, index divisions and LDS round trips (profiles/r02_generic_250_sq.json:
// as many SALU as VALU instructions in the column pass).  For lengths whose prime factors are <= 31
// (fft_smooth.hpp) this file instantiates the same three per-iteration kernels with the plan fixed at
// compile time -- 2 passes for most image sizes (250 = 25 x 10, 480 = 24 x 20, 640 = 32 x 20), the first
// pass loading global memory and the last storing it, so a transform touches LDS (P - 1) times:
//   sm::column_kernel<N>    dim-2 FFT, x Ct (the x-update C / (MN), ops.jl:86), IFFT; the forward's
//                           last pass and the reversed inverse plan's first pass share registers
//   sm::line_inv_kernel<M>  two real lines per complex M-point IFFT (Hermitian extension) -> x
//   sm::line_upd_kernel<M>  s = Dx + clip(s_old), w = z - u, v = H^T y + rho D^T w (ops.jl:169-173),
//                           rFFT of two real lines per complex transform -> half spectra
// Layout (identical to admm_generic.hip, so the one-off PREP kernels, the isotropic kernels and the
// adjoint keep working on the same buffers): spectra [plane][line j][bin k], H = M/2 + 1 bins per line;
// x, s, H^T y [plane][(channel)][j][i].
#include <hip/hip_runtime.h>

#include "fft_smooth.hpp"
#include "smooth_api.hpp"

namespace admm {
namespace sm {

// XCD-aware block order (same bijection as admm_kernels.hip xcd_block): workgroups are dealt
// round-robin over the 8 XCDs; the remap gives each XCD a contiguous run of logical blocks, so blocks
// that share 128-B lines (neighbouring column blocks, the halo lines of line blocks) share an L2.
struct Blk {
    int x, y;
};
__device__ __forceinline__ Blk xcd_block() {
    const unsigned nx = gridDim.x, n = nx * gridDim.y;
    const unsigned orig = blockIdx.x + nx * blockIdx.y;
    const unsigned q = n / 8, r = n % 8, g = orig % 8;
    const unsigned id = (g < r ? g * (q + 1) : r * (q + 1) + (g - r) * q) + orig / 8;
    return {(int)(id % nx), (int)(id / nx)};
}

__device__ __forceinline__ float clipf(float s, float tau) { return fminf(fmaxf(s, -tau), tau); }
// w = z - u for z = ST(s, tau), u = s - z  (ops.jl:9, :171-173)
__device__ __forceinline__ float prox_w(float s, float tau) { return fabsf(s) > tau ? s - copysignf(2.0f * tau, s) : -s; }

// ---- block shapes (host and device agree through these) ---------------------------------------------
constexpr int kNT = 256;
// radix caps: line transforms 16 (more passes but fewer live registers: 250^2 line passes 3.21 -> 2.95 ms
// per solve, 480 x 640 3.90 -> 3.63), column transforms 32 (a smaller cap did not help them)
constexpr int kLineR = 16, kColR = 32;
#ifndef SM_UPD_U
#define SM_UPD_U 8   // strides of loads in flight per thread in the update's elementwise phase
#endif
// column blocks: KB spectral columns (a power of two, <= 16) with the LDS buffer <= 48 KiB; the
// per-column stride FS makes the KB columns x (32 / KB) butterflies of a 32-lane group hit distinct banks
constexpr int col_fs(int NN, int KB) {
    int fs = NN;
    while (fs % 32 != (32 / KB) % 32) ++fs;
    return fs;
}
#ifndef SM_COL_KBMAX
#define SM_COL_KBMAX 16
#endif
#ifndef SM_COL_LDS_KB
#define SM_COL_LDS_KB 48
#endif
constexpr int col_kb(int NN) {
    int kb = SM_COL_KBMAX;
    while (kb > 1 && kb * col_fs(NN, kb) * 8 > SM_COL_LDS_KB * 1024) kb /= 2;
    return kb;
}
// line blocks: TG lines = 2 NP (NP paired complex transforms), enough that the widest pass has about NT
// butterflies, at most 16 lines and 32 KiB of transform buffer
template <int MM>
constexpr int line_np() {
    int np = (kNT + SP<MM, true, kLineR>::max_q() - 1) / SP<MM, true, kLineR>::max_q();
    if (np > 8) np = 8;
    while (np > 1 && np * MM * 8 > 32 * 1024) --np;
    return np;
}

// ---- dim-2 pass --------------------------------------------------------------------------------------
template <int NN, bool ASC>
struct KB_Q {
    static constexpr int q = col_kb(NN) * SP<NN, ASC, kColR>::max_q();
};
// MUL 0: x cs * Ct (the x-update C / (MN), ops.jl:86); 1: x Gt = conj(Sigma_c) / (MN) (H^T, PREP)
// threads per column block: enough for the widest pass's butterflies (KB x Q), in whole waves, <= kNT
#ifndef SM_COL_NT_FIT
#define SM_COL_NT_FIT 1
#endif
template <int NN, bool ASC>
constexpr int col_nt() {
    if (!SM_COL_NT_FIT) return kNT;
    const int q = KB_Q<NN, ASC>::q;
    const int nt = 64 * ((q + 63) / 64);
    return nt < kNT ? nt : kNT;
}
template <int NN, bool ASC, int MUL>
__global__ __launch_bounds__((col_nt<NN, ASC>())) void column_kernel(const float2* __restrict__ src, float2* __restrict__ dst,
                                                     const float* __restrict__ Ct, const float2* __restrict__ Gt,
                                                     const float2* __restrict__ twN, int H, float cs,
                                                     const float2* __restrict__ yh = nullptr) {
    // yh (not NULL): Y_h = F(H^T y), [plane][kj][k], added to the forward spectrum before the multiply (H^T y in
    // the spectral domain, as admm_generic.hip column_kernel mode 16)
    constexpr int KB = col_kb(NN), FS = col_fs(NN, KB), NT = col_nt<NN, ASC>();
    using S = SP<NN, ASC, kColR>;
    constexpr int P = S::P;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float2* tw = reinterpret_cast<float2*>(smem_raw);
    float2* buf = tw + NN;
    const Blk b = xcd_block();
    const int plane = b.y, k0 = b.x * KB;
    const int kc = min(KB, H - k0);
    const size_t po = (size_t)plane * NN * H + k0;
    const float2* gs = src + po;
    float2* gd = dst + po;
    const float* cp = Ct + k0;
    const float2* gp = Gt + k0;
    const float2* yp = yh ? yh + po : nullptr;
    // the multiplier of bin kj of this block's column c
    auto mul = [&](int c, int kj, float2 v) {
        if constexpr (MUL == 0) return cscale(v, cs * cp[(size_t)kj * H + c]);
        else return cmul(v, gp[(size_t)kj * H + c]);
    };
    for (int t = threadIdx.x; t < NN; t += NT) tw[t] = twN[t];
    auto gload = [&](int c, int n) { return c < kc ? gs[(size_t)n * H + c] : make_float2(0.f, 0.f); };
    auto gstore = [&](int c, int n, float2 v) {
        if (c < kc) gd[(size_t)n * H + c] = v;
    };
    if constexpr (P == 1) {
        for (int c = threadIdx.x; c < kc; c += NT) {
            float2 v[NN];
#pragma unroll
            for (int n = 0; n < NN; ++n) v[n] = gload(c, n);
            dftR<NN, false>(v);
#pragma unroll
            for (int n = 0; n < NN; ++n) v[n] = mul(c, n, yp ? cadd(v[n], yp[(size_t)n * H + c]) : v[n]);
            dftR<NN, true>(v);
#pragma unroll
            for (int n = 0; n < NN; ++n) gstore(c, n, v[n]);
        }
    } else {
        const Lds<FS> bl{buf};
        // forward passes 0 .. P-2 (pass 0 has no twiddles: tw is ready after its barrier)
        plan_spass<NN, 0, false, false, NT, KB, false, false, ASC, kColR>(KB, tw, gload, bl);
        __syncthreads();
        if constexpr (P >= 3) {
            plan_spass<NN, 1, false, false, NT, KB, false, true, ASC, kColR>(KB, tw, bl, bl);
            __syncthreads();
        }
        if constexpr (P >= 4) {
            plan_spass<NN, 2, false, false, NT, KB, false, true, ASC, kColR>(KB, tw, bl, bl);
            __syncthreads();
        }
        // forward last pass (radix R, Ns = Q: butterfly j outputs bins j + r Q) -> x Ct -> first pass of the
        // reversed inverse plan (radix R, Ns = 1: reads exactly j + r Q), in registers
        {
            constexpr int R = S::template radix<false>(P - 1);
            constexpr int Q = NN / R;
            constexpr int NR = (KB * Q + NT - 1) / NT;
            float2 v[NR][R];
#pragma unroll
            for (int u = 0; u < NR; ++u) {
                const int idx = (int)threadIdx.x + u * NT;
                if (idx < KB * Q) {
                    const int f = idx % KB, j = idx / KB;
#pragma unroll
                    for (int r = 0; r < R; ++r) v[u][r] = buf[f * FS + j + r * Q];
                }
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < NR; ++u) {
                const int idx = (int)threadIdx.x + u * NT;
                if (idx < KB * Q) {
                    const int f = idx % KB, j = idx / KB;
#pragma unroll
                    for (int r = 1; r < R; ++r) v[u][r] = cmul(v[u][r], tw[r * j]);
                    dftR<R, false>(v[u]);
                    if (f < kc) {
                        if (yp) {
#pragma unroll
                            for (int r = 0; r < R; ++r) v[u][r] = cadd(v[u][r], yp[(size_t)(j + r * Q) * H + f]);
                        }
#pragma unroll
                        for (int r = 0; r < R; ++r) v[u][r] = mul(f, j + r * Q, v[u][r]);
                    }
                    dftR<R, true>(v[u]);
#pragma unroll
                    for (int r = 0; r < R; ++r) buf[f * FS + j * R + r] = v[u][r];
                }
            }
        }
        __syncthreads();
        if constexpr (P >= 4) {
            plan_spass<NN, 1, true, true, NT, KB, false, true, ASC, kColR>(KB, tw, bl, bl);
            __syncthreads();
        }
        if constexpr (P >= 3) {
            plan_spass<NN, P - 2, true, true, NT, KB, false, true, ASC, kColR>(KB, tw, bl, bl);
            __syncthreads();
        }
        plan_spass<NN, P - 1, true, true, NT, KB, false, false, ASC, kColR>(KB, tw, bl, gstore);
    }
}

// Block-stride loop over [0, total) that issues the global loads of U consecutive strides before any of
// their uses (a loop whose body loads global memory and stores LDS otherwise pays one memory latency per
// stride: the compiler does not move loads across the LDS stores).
template <int U, class Load, class Use>
__device__ __forceinline__ void batched(int total, Load&& load, Use&& use) {
    using V = decltype(load(0));
    for (int b0 = threadIdx.x; b0 < total; b0 += U * kNT) {
        V v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = b0 + u * kNT;
            if (i < total) v[u] = load(i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = b0 + u * kNT;
            if (i < total) use(i, v[u]);
        }
    }
}

// ---- dim-1 inverse: half spectra -> real lines (x) ----------------------------------------------------
// The block's T spectrum rows are one contiguous run: every thread copies part of it to LDS (batched
// loads), then the first FFT pass forms Z = X_2f + i X_2f+1 with the Hermitian extensions from LDS (in
// place over the staged rows) and the last pass writes the two real lines.
template <int MM>
__global__ __launch_bounds__(kNT) void line_inv_kernel(const float2* __restrict__ spec, float* __restrict__ dst,
                                                       const float2* __restrict__ twM, int N) {
    constexpr int H = MM / 2 + 1, NP = line_np<MM>(), TG = 2 * NP;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float2* tw = reinterpret_cast<float2*>(smem_raw);
    float2* A = tw + MM;   // staged rows (TG x H), then the transforms (NP x MM), in place
    const Blk b = xcd_block();
    const int plane = b.y, j0 = b.x * TG;
    const int T = min(TG, N - j0);   // the last block of a plane may be ragged
    const float2* sp = spec + ((size_t)plane * N + j0) * H;
    float* dp = dst + ((size_t)plane * N + j0) * MM;
    for (int t = threadIdx.x; t < MM; t += kNT) tw[t] = twM[t];
    batched<8>(T * H, [&](int idx) { return sp[idx]; }, [&](int idx, float2 v) { A[idx] = v; });
    __syncthreads();
    // Z = X_2f + i X_2f+1 with Hermitian extensions; DC and Nyquist taken real (what the real part of a
    // single line's inverse keeps) -> z = x_2f + i x_2f+1
    auto zload = [&](int f, int k) {
        const float2* sa = A + (2 * f) * H;
        const bool lo = k < H;
        float2 ev = lo ? sa[k] : cconj(sa[MM - k]);
        float2 od = make_float2(0.f, 0.f);
        if (2 * f + 1 < T) od = lo ? sa[H + k] : cconj(sa[H + MM - k]);
        if (k == 0 || 2 * k == MM) ev.y = od.y = 0.0f;
        return make_float2(ev.x - od.y, ev.y + od.x);
    };
    auto xstore = [&](int f, int n, float2 v) {
        dp[(size_t)(2 * f) * MM + n] = v.x;
        if (2 * f + 1 < T) dp[(size_t)(2 * f + 1) * MM + n] = v.y;
    };
    splan<MM, true, kNT, NP, true, MM, true, false, true, kLineR>((T + 1) / 2, tw, A, zload, xstore);
}

// ---- dim-1 forward: real lines (y, H^T y) -> half spectra (PREP) ---------------------------------------
// The block's T rows are contiguous: all threads load them as packed pairs (line 2p real part, 2p + 1
// imaginary), then the FFT runs in place and the half spectra are separated (as in the update kernel).
template <int MM>
__global__ __launch_bounds__(kNT) void line_fwd_kernel(const float* __restrict__ src, float2* __restrict__ spec,
                                                       const float2* __restrict__ twM, int N) {
    constexpr int H = MM / 2 + 1, NP = line_np<MM>(), TG = 2 * NP;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float2* tw = reinterpret_cast<float2*>(smem_raw);
    float2* A = tw + MM;
    float* Af = reinterpret_cast<float*>(A);
    const Blk b = xcd_block();
    const int plane = b.y, j0 = b.x * TG;
    const int T = min(TG, N - j0);
    const float* sp = src + ((size_t)plane * N + j0) * MM;
    for (int t = threadIdx.x; t < MM; t += kNT) tw[t] = twM[t];
    batched<8>(T * MM, [&](int idx) { return sp[idx]; }, [&](int idx, float v) {
        const int t = idx / MM, i = idx - t * MM;
        Af[2 * ((t >> 1) * MM + i) + (t & 1)] = v;
    });
    if (T & 1)
        for (int i = threadIdx.x; i < MM; i += kNT) A[(T >> 1) * MM + i].y = 0.0f;
    __syncthreads();
    const Lds<MM> al{A};
    splan<MM, false, kNT, NP, true, MM, true, true, true, kLineR>((T + 1) / 2, tw, A, al, al);
    __syncthreads();
    float2* dp = spec + ((size_t)plane * N + j0) * H;
    for (int idx = threadIdx.x; idx < T * H; idx += kNT) {
        const int t = idx / H, k = idx - t * H;
        const float2* Z = A + (t >> 1) * MM;
        const float2 z = Z[k], zm = cconj(Z[k == 0 ? 0 : MM - k]);
        dp[idx] = (t & 1) ? make_float2(0.5f * (z.y - zm.y), -0.5f * (z.x - zm.x))
                          : make_float2(0.5f * (z.x + zm.x), 0.5f * (z.y + zm.y));
    }
}

// ---- dim-1 update + forward (iterations 1 .. K-1, anisotropic) -------------------------------------
// Phase 1, every pixel of rows j0 .. j0+T (row j0+T: the halo below, channel 0 only) in parallel with
// batched loads: s = D x + clip(s_old), s_new stored, w = z - u (both channels) to LDS.  H^T y for the
// first FFT pass is loaded before phase 1 (in flight meanwhile).  Phase 2 = the first forward pass: it
// forms v = H^T y + rho D^T w for lines 2f (real part) and 2f+1 (imaginary) straight from the w rows, and
// writes the transforms over them (all reads before a barrier).  Then the remaining passes in place, and
// the half spectra separated: X_2p = (Z + conj Z(-k)) / 2, X_2p+1 = (Z - conj Z(-k)) / (2i).
#ifndef SM_UPD_LDS_KB
#define SM_UPD_LDS_KB 40
#endif
template <int MM>
constexpr int upd_np() {   // paired transforms per update block: w rows (2 TG + 1) x MM floats <= 40 KiB
    int np = line_np<MM>();
    while (np > 1 && (4 * np + 1) * MM * 4 > SM_UPD_LDS_KB * 1024) --np;
    return np;
}
template <int MM>
__global__ __launch_bounds__(kNT) void line_upd_kernel(const float* __restrict__ x, const float* __restrict__ s_old,
                                                       float* __restrict__ s_new, const float* __restrict__ hty,
                                                       float2* __restrict__ spec, const float2* __restrict__ twM,
                                                       int N, const float* __restrict__ prm, int first) {
    constexpr int H = MM / 2 + 1, NP = upd_np<MM>(), TG = 2 * NP;
    using S = SP<MM, true, kLineR>;
    constexpr int P = S::P;
    constexpr int R0 = S::template radix<false>(0), Q0 = MM / R0;
    constexpr int NR0 = (NP * Q0 + kNT - 1) / kNT;
    const float tau = prm[0], rho = prm[1];
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float2* tw = reinterpret_cast<float2*>(smem_raw);
    float* W0 = reinterpret_cast<float*>(tw + MM);   // TG + 1 rows
    float* W1 = W0 + (TG + 1) * MM;                  // TG rows
    float2* A = reinterpret_cast<float2*>(W0);       // NP transforms over the w rows
    const Blk b = xcd_block();
    const int plane = b.y, j0 = b.x * TG;
    const int T = min(TG, N - j0);
    const int np = (T + 1) / 2;
    const size_t MN = (size_t)MM * N;
    const float* xp = x + (size_t)plane * MN;
    const float* so = s_old + (size_t)plane * 2 * MN;
    float* sn = s_new + (size_t)plane * 2 * MN;
    // hty NULL: H^T y enters spectrally (the runtime column kernel's mode 16), v = rho D^T w here
    const float* hp = hty ? hty + ((size_t)plane * N + j0) * MM : nullptr;
    for (int t = threadIdx.x; t < MM; t += kNT) tw[t] = twM[t];
    // H^T y of this thread's first-pass points (lines 2f, 2f+1 at n = j + r Q0)
    float2 hv[NR0][R0];
#pragma unroll
    for (int u = 0; u < NR0; ++u) {
        const int idx = (int)threadIdx.x + u * kNT;
        if (idx < np * Q0) {
            const int f = idx / Q0, j = idx - f * Q0;
            const bool odd = 2 * f + 1 < T;
#pragma unroll
            for (int r = 0; r < R0; ++r) {
                const int n = j + r * Q0;
                hv[u][r].x = hp ? hp[(size_t)(2 * f) * MM + n] : 0.0f;
                hv[u][r].y = (hp && odd) ? hp[(size_t)(2 * f + 1) * MM + n] : 0.0f;
            }
        }
    }
    // phase 1
    struct UpdIn {
        float xc, xu, xl, a0, a1;
    };
    batched<SM_UPD_U>((T + 1) * MM, [&](int idx) {
        const int t = idx / MM, i = idx - t * MM;
        int jj = j0 + t;
        if (jj >= N) jj -= N;
        const int jp = jj == 0 ? N - 1 : jj - 1;
        const size_t o = (size_t)jj * MM + i;
        UpdIn r;
        r.xc = xp[o];
        r.xu = xp[(size_t)jp * MM + i];
        r.xl = t < T ? xp[(size_t)jj * MM + (i == 0 ? MM - 1 : i - 1)] : 0.0f;
        r.a0 = first ? 0.0f : so[o];
        r.a1 = (first || t >= T) ? 0.0f : so[MN + o];
        return r;
    }, [&](int idx, const UpdIn& r) {
        const int t = idx / MM;
        const float s0 = (r.xc - r.xu) + clipf(r.a0, tau);
        W0[idx] = prox_w(s0, tau);
        if (t < T) {
            const int i = idx - t * MM;
            const size_t o = (size_t)(j0 + t) * MM + i;
            const float s1 = (r.xc - r.xl) + clipf(r.a1, tau);
            W1[idx] = prox_w(s1, tau);
            sn[o] = s0;
            sn[MN + o] = s1;
        }
    });
    __syncthreads();
    // phase 2: first forward pass (radix R0, Ns = 1) fed by v = H^T y + rho D^T w, written over the w rows
    {
        float2 v[NR0][R0];
#pragma unroll
        for (int u = 0; u < NR0; ++u) {
            const int idx = (int)threadIdx.x + u * kNT;
            if (idx < np * Q0) {
                const int f = idx / Q0, j = idx - f * Q0;
                const bool odd = 2 * f + 1 < T;
                const float* w0a = W0 + (2 * f) * MM;
                const float* w1a = W1 + (2 * f) * MM;
#pragma unroll
                for (int r = 0; r < R0; ++r) {
                    const int n = j + r * Q0, n1 = n + 1 == MM ? 0 : n + 1;
                    const float da = (w0a[n] - w0a[MM + n]) + (w1a[n] - w1a[n1]);
                    float db = 0.0f;
                    if (odd) db = (w0a[MM + n] - w0a[2 * MM + n]) + (w1a[MM + n] - w1a[MM + n1]);
                    v[u][r] = make_float2(fmaf(rho, da, hv[u][r].x), odd ? fmaf(rho, db, hv[u][r].y) : 0.0f);
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < NR0; ++u) {
            const int idx = (int)threadIdx.x + u * kNT;
            if (idx < np * Q0) {
                const int f = idx / Q0, j = idx - f * Q0;
                dftR<R0, false>(v[u]);
#pragma unroll
                for (int r = 0; r < R0; ++r) A[f * MM + j * R0 + r] = v[u][r];
            }
        }
    }
    __syncthreads();
    const Lds<MM> al{A};
    if constexpr (P >= 3) {
        plan_spass<MM, 1, false, false, kNT, NP, true, true, true, kLineR>(np, tw, al, al);
        __syncthreads();
    }
    if constexpr (P >= 4) {
        plan_spass<MM, 2, false, false, kNT, NP, true, true, true, kLineR>(np, tw, al, al);
        __syncthreads();
    }
    if constexpr (P >= 2) {
        plan_spass<MM, P - 1, false, false, kNT, NP, true, true, true, kLineR>(np, tw, al, al);
        __syncthreads();
    }
    float2* dp = spec + ((size_t)plane * N + j0) * H;
    for (int idx = threadIdx.x; idx < T * H; idx += kNT) {
        const int t = idx / H, k = idx - t * H;
        const float2* Z = A + (t >> 1) * MM;
        const float2 z = Z[k], zm = cconj(Z[k == 0 ? 0 : MM - k]);
        dp[idx] = (t & 1) ? make_float2(0.5f * (z.y - zm.y), -0.5f * (z.x - zm.x))
                          : make_float2(0.5f * (z.x + zm.x), 0.5f * (z.y + zm.y));
    }
}

// ---- host side: instance tables ---------------------------------------------------------------------
// Lengths compiled here (any of them on either side, independently): common image sizes whose prime
// factors are <= 31, plus the powers of two the tuned path does not take (2048, 4096; and any power of
// two paired with a non-power-of-two other side).
#define SM_LENGTHS(X)                                                                                     \
    X(64) X(96) X(100) X(120) X(128) X(144) X(160) X(192) X(200) X(240) X(250) X(256) X(288) X(300) X(320) \
    X(360) X(384) X(400) X(480) X(500) X(512) X(576) X(600) X(640) X(720) X(768) X(800) X(960) X(1000)   \
    X(1024) X(1080) X(1200) X(1280) X(1440) X(1536) X(1920) X(2000) X(2048) X(2560) X(3000) X(4096)

bool has_length(int n) {
#define X(v) \
    if (n == v) return true;
    SM_LENGTHS(X)
#undef X
    return false;
}

int line_lines(int M) {
#define X(v) \
    if (M == v) return 2 * line_np<v>();
    SM_LENGTHS(X)
#undef X
    return 0;
}
int column_slots(int N) {
#define X(v) \
    if (N == v) return col_kb(v);
    SM_LENGTHS(X)
#undef X
    return 0;
}
size_t line_lds(int M) {
    const int tg = line_lines(M);
    return (size_t)M * 8 + (size_t)tg * (M / 2 + 1) * 8;   // twiddles + staged rows (>= the transforms)
}
int upd_lines(int M) {
#define X(v) \
    if (M == v) return 2 * upd_np<v>();
    SM_LENGTHS(X)
#undef X
    return 0;
}
size_t upd_lds(int M) { return (size_t)M * 8 + (size_t)(2 * upd_lines(M) + 1) * M * 4; }
size_t column_lds(int N) {
    const int kb = column_slots(N);
    return (size_t)N * 8 + (size_t)kb * col_fs(N, kb) * 8;
}

template <typename K>
static void set_lds(K kernel, size_t lds) {
    if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

// Column plan order per length (decreasing radices unless listed): measured on MI355X with
// tools/col_order_sweep.py (K = 25 column passes, 1 x MI355X); e.g. 250: 10 x 25 0.99 ms vs 25 x 10 1.44,
// 480: 24 x 20 1.39 ms vs 20 x 24 1.70.  ADMM_OPT_SMOOTH = 2 / 3 force increasing / decreasing (sweeps).
#define SM_COL_ASC_LENGTHS(X) X(192) X(200) X(250) X(300) X(320) X(360) X(400) X(500) X(600) X(720) X(1200) X(2000)
bool column_asc(int N, int mode) {
    if (mode == 2) return true;
    if (mode == 3) return false;
#define X(v) \
    if (N == v) return true;
    SM_COL_ASC_LENGTHS(X)
#undef X
    return false;
}

int launch_column(int M, int N, size_t planes, hipStream_t s, const float2* src, float2* dst, const float* Ct,
                  const float2* Gt, const float2* twN, float cs, int mul, int mode, const float2* yh) {
    const int H = M / 2 + 1;
    const bool asc = column_asc(N, mode);
#define X(v)                                                                                               \
    if (N == v) {                                                                                          \
        constexpr int kb = col_kb(v);                                                                      \
        const size_t lds = column_lds(v);                                                                  \
        const dim3 g((H + kb - 1) / kb, (unsigned)planes);                                                 \
        if (mul) {                                                                                         \
            set_lds(column_kernel<v, false, 1>, lds);                                                      \
            column_kernel<v, false, 1><<<g, col_nt<v, false>(), lds, s>>>(src, dst, Ct, Gt, twN, H, cs, yh);              \
        } else if (asc) {                                                                                  \
            set_lds(column_kernel<v, true, 0>, lds);                                                       \
            column_kernel<v, true, 0><<<g, col_nt<v, true>(), lds, s>>>(src, dst, Ct, Gt, twN, H, cs, yh);               \
        } else {                                                                                           \
            set_lds(column_kernel<v, false, 0>, lds);                                                      \
            column_kernel<v, false, 0><<<g, col_nt<v, false>(), lds, s>>>(src, dst, Ct, Gt, twN, H, cs, yh);              \
        }                                                                                                  \
        return 0;                                                                                          \
    }
    SM_LENGTHS(X)
#undef X
    return -1;
}

int launch_line_fwd(int M, int N, size_t planes, hipStream_t s, const float* src, float2* spec, const float2* twM) {
#define X(v)                                                                                                  \
    if (M == v) {                                                                                             \
        const int tg = 2 * line_np<v>();                                                                      \
        const size_t lds = line_lds(v);                                                                       \
        set_lds(line_fwd_kernel<v>, lds);                                                                     \
        line_fwd_kernel<v><<<dim3((N + tg - 1) / tg, (unsigned)planes), kNT, lds, s>>>(src, spec, twM, N);   \
        return 0;                                                                                             \
    }
    SM_LENGTHS(X)
#undef X
    return -1;
}

int launch_line_inv(int M, int N, size_t planes, hipStream_t s, const float2* spec, float* dst, const float2* twM) {
#define X(v)                                                                                                  \
    if (M == v) {                                                                                             \
        const int tg = 2 * line_np<v>();                                                                      \
        const size_t lds = line_lds(v);                                                                       \
        set_lds(line_inv_kernel<v>, lds);                                                                     \
        line_inv_kernel<v><<<dim3((N + tg - 1) / tg, (unsigned)planes), kNT, lds, s>>>(spec, dst, twM, N);   \
        return 0;                                                                                             \
    }
    SM_LENGTHS(X)
#undef X
    return -1;
}

int launch_line_upd(int M, int N, size_t planes, hipStream_t s, const float* x, const float* s_old, float* s_new,
                    const float* hty, float2* spec, const float2* twM, const float* prm, int first) {
#define X(v)                                                                                                \
    if (M == v) {                                                                                           \
        const int tg = 2 * upd_np<v>();                                                                     \
        const size_t lds = upd_lds(v);                                                                      \
        set_lds(line_upd_kernel<v>, lds);                                                                   \
        line_upd_kernel<v><<<dim3((N + tg - 1) / tg, (unsigned)planes), kNT, lds, s>>>(x, s_old, s_new, hty, \
                                                                                       spec, twM, N, prm, first); \
        return 0;                                                                                           \
    }
    SM_LENGTHS(X)
#undef X
    return -1;
}

}  // namespace sm
}  // namespace admm
