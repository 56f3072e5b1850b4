// admm_generic.hip -- the solve for shapes outside the power-of-two kernels' support matrix.
//
// The reference accepts any M x N (FFTW / CUFFT plans, /root/reference/src/ops/ops.jl:26,35-36,86 and
// :108,117-118,168), e.g. 96 x 96 demos or 480 x 640 photographs.  The tuned path (admm_kernels.hip,
// plane_kernel.hip) is specialised for powers of two; this file keeps the same 2-pass structure with
// RUNTIME lengths:
//   * mixed-radix Stockham FFTs staged in LDS, radix 8/4/2/3/5 butterflies in registers and a direct
//     DFT for any other prime factor (so every length works; 2-3-5-smooth lengths are the fast case);
//   * dim-1 (contiguous, real) transforms as complex FFTs of two real lines at once (real and
//     imaginary part), keeping bins 0..M/2 of each (the rfft half spectrum, ops.jl:86) -- M may be odd;
//   * per iteration: GEN_COLUMN (dim-2 FFT, x C/(MN), inverse) -> GEN_LINE_INV (x to HBM) ->
//     GEN_LINE_UPD (D, prox, dual, D^T, + H^T y, dim-1 FFT) -- or the iso triple GEN_ISO_A -> ISO_R ->
//     GEN_ISO_B.  x takes one extra HBM round trip compared with the fused line kernel (8 B/px).
// Spectrum layout: [plane][line j][bin k], H = M/2 + 1 bins per line (k fastest).
#include <hip/hip_runtime.h>

namespace admm {
namespace gen {

constexpr int kMaxF = 24;
// factorisation of a transform length, applied in this order (built on the host)
struct FPlan {
    int n, nf;
    int r[kMaxF];
};

template <bool INV>
__device__ __forceinline__ float2 twid(const float2* __restrict__ tw, int t) {
    const float2 w = tw[t];   // exp(-2 pi i t / n)
    return INV ? cconj(w) : w;
}
__device__ __forceinline__ float2 mul_i(float2 z) { return make_float2(-z.y, z.x); }

template <bool INV>
__device__ __forceinline__ void dft3(float2& a, float2& b, float2& c) {
    constexpr float c1 = -0.5f;
    constexpr float s1 = INV ? 0.866025403784438647f : -0.866025403784438647f;
    const float2 t = cadd(b, c), d = cscale(csub(b, c), s1);
    const float2 m = make_float2(fmaf(c1, t.x, a.x), fmaf(c1, t.y, a.y));
    a = cadd(a, t);
    b = cadd(m, mul_i(d));
    c = csub(m, mul_i(d));
}

template <bool INV>
__device__ __forceinline__ void dft5(float2 (&x)[5]) {
    constexpr float c1 = 0.309016994374947424f, c2 = -0.809016994374947424f;
    constexpr float sg = INV ? 1.0f : -1.0f;
    constexpr float s1 = sg * 0.951056516295153572f, s2 = sg * 0.587785252292473129f;
    const float2 t1 = cadd(x[1], x[4]), t2 = cadd(x[2], x[3]);
    const float2 d1 = csub(x[1], x[4]), d2 = csub(x[2], x[3]);
    const float2 m1 = make_float2(x[0].x + c1 * t1.x + c2 * t2.x, x[0].y + c1 * t1.y + c2 * t2.y);
    const float2 m2 = make_float2(x[0].x + c2 * t1.x + c1 * t2.x, x[0].y + c2 * t1.y + c1 * t2.y);
    const float2 e1 = mul_i(make_float2(s1 * d1.x + s2 * d2.x, s1 * d1.y + s2 * d2.y));
    const float2 e2 = mul_i(make_float2(s2 * d1.x - s1 * d2.x, s2 * d1.y - s1 * d2.y));
    x[0] = cadd(x[0], cadd(t1, t2));
    x[1] = cadd(m1, e1);
    x[4] = csub(m1, e1);
    x[2] = cadd(m2, e2);
    x[3] = csub(m2, e2);
}

// n / d for 0 <= n < 2^22, d >= 1 (exact): a v_rcp_f32 estimate is within 1 of the quotient there, and
// one correction step fixes it -- a handful of VALU against ~30 for the compiler's integer-division
// sequence (d is a runtime plan length, so there is no constant to divide by).  The reciprocal is loop
// invariant at every call site.
__device__ __forceinline__ int fdiv(int n, int d) {
    const int q = (int)((float)n * __builtin_amdgcn_rcpf((float)d));
    const int r = n - q * d;
    return q + (r >= d) - (r < 0);
}

// one radix-R butterfly of a Stockham pass: src[j + a q] (a < R) twiddled by W_{Ns R}^{a k}, DFT_R,
// to dst[(j / Ns) Ns R + k + c Ns]
template <int R, bool INV>
__device__ __forceinline__ void bfly(const float2* __restrict__ src, float2* __restrict__ dst, int j, int q, int Ns,
                                     int tstep, const float2* __restrict__ tw) {
    const int jn = fdiv(j, Ns);
    const int k = j - jn * Ns;
    float2 v[R];
#pragma unroll
    for (int a = 0; a < R; ++a) {
        v[a] = src[j + a * q];
        if (a > 0 && k > 0) v[a] = cmul(v[a], twid<INV>(tw, a * k * tstep));
    }
    if constexpr (R == 3) {
        dft3<INV>(v[0], v[1], v[2]);
    } else if constexpr (R == 5) {
        dft5<INV>(v);
    } else {
        dft<R, INV>(v);
    }
    const int base = jn * Ns * R + k;
#pragma unroll
    for (int c = 0; c < R; ++c) dst[base + c * Ns] = v[c];
}

// any radix (prime factors other than 2, 3, 5): direct O(R^2) evaluation from LDS
template <bool INV>
__device__ __forceinline__ void bfly_any(const float2* __restrict__ src, float2* __restrict__ dst, int j, int q,
                                         int Ns, int R, int n, int tstep, const float2* __restrict__ tw) {
    const int jn = fdiv(j, Ns);
    const int k = j - jn * Ns;
    const int base = jn * Ns * R + k;
    const int rstep = n / R;
    for (int c = 0; c < R; ++c) {
        float2 acc = make_float2(0.f, 0.f);
        for (int a = 0; a < R; ++a) {
            float2 x = src[j + a * q];
            if (a > 0 && k > 0) x = cmul(x, twid<INV>(tw, a * k * tstep));
            acc = cadd(acc, cmul(x, twid<INV>(tw, ((a * c) % R) * rstep)));
        }
        dst[base + c * Ns] = acc;
    }
}

// LDS hand-off between the lanes of one wave: a wave's LDS instructions execute in order; the fences keep
// the compiler from moving this pass's loads above the previous pass's stores.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int R, bool INV>
__device__ __forceinline__ void wave_pass(const float2* __restrict__ src, float2* __restrict__ dst, int lane, int q,
                                          int Ns, int tstep, const float2* __restrict__ tw) {
    for (int j = lane; j < q; j += 64) bfly<R, INV>(src, dst, j, q, Ns, tstep, tw);
}

// cnt transforms of length pl.n at a[t * stride ...]; ping-pong with b; returns the buffer holding the
// result.  One WAVE per transform (transform t on wave t mod nwaves): the passes of a transform hand off
// through LDS with wave-level ordering only, so the block's waves run their transforms without block
// barriers between passes (a 250-point line is 4 passes of 50..125 butterflies: per-pass block barriers
// were most of its time).  The caller synchronises before (input ready); this ends with a block barrier.
// GEN_WAVE_FFT 1 (default): per-wave passes when every wave has a transform and transforms are long
// enough to fill a wave's lanes (n >= 128), else block-wide passes; 0: always block-wide; 2: always per-wave.
// Measured (1x MI355X, K=25, tools/gen_variants.sh): per-wave 250^2 40.3k img/s vs block-wide 36.8k; 96^2
// 182k vs 225k (12..48-butterfly passes), 2048^2 206 vs 292 (one transform per column block).
#ifndef GEN_WAVE_FFT
#define GEN_WAVE_FFT 1
#endif
template <bool INV>
__device__ float2* fft(float2* a, float2* b, int cnt, int stride, const FPlan& pl, const float2* __restrict__ tw) {
    const int n = pl.n;
    const bool wave_mode = GEN_WAVE_FFT == 2 || (GEN_WAVE_FFT == 1 && cnt >= (int)(blockDim.x >> 6) && n >= 128);
    if (!wave_mode) {
    // block-wide passes (one block barrier per pass): every thread takes butterflies of every transform
    int Ns = 1;
    for (int p = 0; p < pl.nf; ++p) {
        const int R = pl.r[p];
        const int q = n / R;
        const int tstep = n / (Ns * R);
        for (int idx = threadIdx.x; idx < cnt * q; idx += blockDim.x) {
            const int line = fdiv(idx, q), j = idx - line * q;
            const float2* src = a + (size_t)line * stride;
            float2* dst = b + (size_t)line * stride;
            switch (R) {
                case 2: bfly<2, INV>(src, dst, j, q, Ns, tstep, tw); break;
                case 3: bfly<3, INV>(src, dst, j, q, Ns, tstep, tw); break;
                case 4: bfly<4, INV>(src, dst, j, q, Ns, tstep, tw); break;
                case 5: bfly<5, INV>(src, dst, j, q, Ns, tstep, tw); break;
                case 8: bfly<8, INV>(src, dst, j, q, Ns, tstep, tw); break;
                default: bfly_any<INV>(src, dst, j, q, Ns, R, n, tstep, tw); break;
            }
        }
        __syncthreads();
        Ns *= R;
        float2* t = a;
        a = b;
        b = t;
    }
    return a;
    }
    const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    for (int f = threadIdx.x >> 6; f < cnt; f += nw) {
        const float2* src = a + (size_t)f * stride;
        float2* dst = b + (size_t)f * stride;
        int Ns = 1;
        for (int p = 0; p < pl.nf; ++p) {
            const int R = pl.r[p];
            const int q = n / R;
            const int tstep = n / (Ns * R);
            switch (R) {
                case 2: wave_pass<2, INV>(src, dst, lane, q, Ns, tstep, tw); break;
                case 3: wave_pass<3, INV>(src, dst, lane, q, Ns, tstep, tw); break;
                case 4: wave_pass<4, INV>(src, dst, lane, q, Ns, tstep, tw); break;
                case 5: wave_pass<5, INV>(src, dst, lane, q, Ns, tstep, tw); break;
                case 8: wave_pass<8, INV>(src, dst, lane, q, Ns, tstep, tw); break;
                default:
                    for (int j = lane; j < q; j += 64) bfly_any<INV>(src, dst, j, q, Ns, R, n, tstep, tw);
                    break;
            }
            wave_sync();
            Ns *= R;
            const float2* t = dst;
            dst = const_cast<float2*>(src);
            src = t;
        }
    }
    __syncthreads();
    return (pl.nf & 1) ? b : a;
}

// Block-stride loop over [0, total) that issues the global loads of U consecutive strides before any of
// their uses.  A plain loop whose body loads global memory and stores LDS runs one load latency per
// stride (the compiler does not pipeline across the LDS stores); SQ counters of the 250 x 250 line
// kernels showed their waves waiting most of their lifetime.
template <int U, class Load, class Use>
__device__ __forceinline__ void batched(int total, Load&& load, Use&& use) {
    using V = decltype(load(0));
    for (int b = threadIdx.x; b < total; b += U * (int)blockDim.x) {
        V v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = b + u * (int)blockDim.x;
            if (i < total) v[u] = load(i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = b + u * (int)blockDim.x;
            if (i < total) use(i, v[u]);
        }
    }
}
constexpr int kU = 4;

__device__ __forceinline__ int wrap(int i, int n) { return i < 0 ? i + n : (i >= n ? i - n : i); }

// The n twiddles copied to LDS at byte offset off of the dynamic LDS (8-B aligned; the host adds 8 n + 8
// bytes): the butterflies read them once per twiddled point, from global memory that is an L1/L2 round
// trip each.  Visible after the caller's next block barrier.
__device__ __forceinline__ const float2* stage_tw(unsigned char* smem, size_t off, const float2* __restrict__ tw, int n) {
    float2* d = reinterpret_cast<float2*>(smem + ((off + 7) & ~size_t(7)));
    for (int i = threadIdx.x; i < n; i += blockDim.x) d[i] = tw[i];
    return d;
}
// Real lines two per complex transform: lines 2p and 2p+1 are the real and imaginary parts of
// transform p (P = ceil(T / 2) transforms instead of T, half the FFT work of a zero-imaginary line).
// pack_real writes value v of line t, pixel i; with T odd, pad_odd zeroes the last transform's
// imaginary part.  store_real_spectra separates the half spectra: X_2p = (Z + conj Z(-k)) / 2,
// X_2p+1 = (Z - conj Z(-k)) / (2i), bins 0..M/2.
__device__ __forceinline__ void pack_real(float2* A, int t, int i, int M, float v) {
    reinterpret_cast<float*>(A)[2 * ((size_t)(t >> 1) * M + i) + (t & 1)] = v;
}
__device__ __forceinline__ void pad_odd(float2* A, int T, int M) {
    if (T & 1)
        for (int i = threadIdx.x; i < M; i += blockDim.x) A[(size_t)(T >> 1) * M + i].y = 0.0f;
}
__device__ __forceinline__ void store_real_spectra(const float2* __restrict__ R, float2* __restrict__ dp, int T, int M) {
    const int H = M / 2 + 1;
    for (int idx = threadIdx.x; idx < T * H; idx += blockDim.x) {
        const int t = fdiv(idx, H), k = idx - t * H;
        const float2* Z = R + (size_t)(t >> 1) * M;
        const float2 z = Z[k], zm = cconj(Z[k == 0 ? 0 : M - k]);
        dp[idx] = (t & 1) ? make_float2(0.5f * (z.y - zm.y), -0.5f * (z.x - zm.x))
                          : make_float2(0.5f * (z.x + zm.x), 0.5f * (z.y + zm.y));
    }
}

__device__ __forceinline__ float clip(float s, float tau) { return fminf(fmaxf(s, -tau), tau); }
__device__ __forceinline__ float phi(float s, float tau) { return fabsf(s) > tau ? s - copysignf(2.0f * tau, s) : -s; }

// real lines -> half spectra (T lines per block, grid (N / T, planes))
__global__ __launch_bounds__(256) void line_fwd_kernel(const float* __restrict__ src, float2* __restrict__ spec,
                                                       const float2* __restrict__ twM, FPlan pM, int N, int Tg) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int M = pM.n, H = M / 2 + 1;
    float2* A = reinterpret_cast<float2*>(smem_raw);
    float2* B = A + (size_t)((Tg + 1) / 2) * M;   // P = ceil(Tg / 2) paired transforms
    const XBlk xb = xcd_block();   // XCD-aware block order (admm_kernels.hip): neighbours share L2 lines
    const int plane = xb.y, j0 = xb.x * Tg;
    const int T = min(Tg, N - j0);   // the last block of a plane may be ragged (gen_nb)
    const float* sp = src + ((size_t)plane * N + j0) * M;
    const float2* tw = stage_tw(smem_raw, (size_t)16 * ((Tg + 1) / 2) * M, twM, M);
    batched<kU>(T * M, [&](int idx) { return sp[idx]; }, [&](int idx, float v) {
        const int t = fdiv(idx, M);
        pack_real(A, t, idx - t * M, M, v);
    });
    pad_odd(A, T, M);
    __syncthreads();
    const float2* R = fft<false>(A, B, (T + 1) / 2, M, pM, tw);
    store_real_spectra(R, spec + ((size_t)plane * N + j0) * H, T, M);
}

// half spectra -> real lines (Hermitian extension, complex inverse, real part; unnormalised)
__global__ __launch_bounds__(256) void line_inv_kernel(const float2* __restrict__ spec, float* __restrict__ dst,
                                                       const float2* __restrict__ twM, FPlan pM, int N, int Tg) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int M = pM.n, H = M / 2 + 1;
    float2* A = reinterpret_cast<float2*>(smem_raw);
    float2* B = A + (size_t)((Tg + 1) / 2) * M;   // P = ceil(Tg / 2) paired transforms
    const XBlk xb = xcd_block();   // XCD-aware block order (admm_kernels.hip): neighbours share L2 lines
    const int plane = xb.y, j0 = xb.x * Tg;
    const int T = min(Tg, N - j0);   // the last block of a plane may be ragged (gen_nb)
    const float2* sp = spec + ((size_t)plane * N + j0) * H;
    const float2* tw = stage_tw(smem_raw, (size_t)16 * ((Tg + 1) / 2) * M, twM, M);
    // two lines per transform: Z = X_2p + i X_2p+1 (Hermitian extensions, DC / Nyquist bins taken real,
    // which is what the real part of one line's inverse keeps) -> z = x_2p + i x_2p+1
    const int P = (T + 1) / 2;
    batched<kU>(P * M, [&](int idx) {
        const int p = fdiv(idx, M), k = idx - p * M;
        const float2* sa = sp + (size_t)(2 * p) * H;
        float2 ev = k < H ? sa[k] : cconj(sa[M - k]);   // line 2p
        float2 od = make_float2(0.0f, 0.0f);             // line 2p + 1
        if (2 * p + 1 < T) od = k < H ? sa[H + k] : cconj(sa[H + M - k]);
        if (k == 0 || 2 * k == M) ev.y = od.y = 0.0f;
        return make_float2(ev.x - od.y, ev.y + od.x);
    }, [&](int idx, float2 v) { A[idx] = v; });
    __syncthreads();
    const float2* R = fft<true>(A, B, P, M, pM, tw);
    float* dp = dst + ((size_t)plane * N + j0) * M;
    for (int idx = threadIdx.x; idx < T * M; idx += blockDim.x) {
        const int t = fdiv(idx, M);
        const float2 v = R[(size_t)(t >> 1) * M + idx - t * M];
        dp[idx] = (t & 1) ? v.y : v.x;
    }
}

// dim-2 transforms of KB spectral columns: FFT_N, x multiplier, IFFT_N (grid (ceil(H / KB), planes)).
//   mode & 3 = 0: x cs * Ct (x-update C / (MN), ops.jl:86 -- and its adjoint A^-1);
//              1: x Gt (H^T: conj(Sigma_c) / (MN));  2: x conj(Gt) (H, y_bar = H Vsum in the adjoint)
//   mode & 4: store the dim-2 spectrum before the multiply to vsave [plane][kj][k] (trajectory, h_bar)
//   mode & 8: Qp[plane][kj][k] += Re(conj(G) V) against vsave (adjoint, h_bar)
//   mode & 16: + yh[plane][kj][k] before the save and the multiply (Y_h = F(H^T y): H^T y enters spectrally)
//   mode & 32: store Y_h = cs x (mode & 3 == 1 and Gt: Gt) x the forward spectrum to yh; no inverse, dst untouched
__global__ __launch_bounds__(256) void column_kernel(const float2* __restrict__ src, float2* __restrict__ dst,
                                                     const float* __restrict__ Ct, const float2* __restrict__ Gt,
                                                     const float2* __restrict__ twN, FPlan pN, int H, int KB,
                                                     int mode, float cs, float2* __restrict__ vsave = nullptr,
                                                     double* __restrict__ Qp = nullptr, float2* __restrict__ yh = nullptr) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int N = pN.n;
    float2* A = reinterpret_cast<float2*>(smem_raw);
    float2* B = A + (size_t)KB * N;
    const XBlk xb = xcd_block();   // XCD-aware block order (admm_kernels.hip): neighbours share L2 lines
    const int plane = xb.y, k0 = xb.x * KB;
    const int kc = min(KB, H - k0);
    const float2* sp = src + (size_t)plane * N * H + k0;
    float2* dp = dst + (size_t)plane * N * H + k0;
    const float2* tw = stage_tw(smem_raw, (size_t)16 * KB * N, twN, N);
    batched<kU>(N * KB, [&](int idx) {
        const int j = fdiv(idx, KB), c = idx - j * KB;
        return c < kc ? sp[(size_t)j * H + c] : make_float2(0.f, 0.f);
    }, [&](int idx, float2 v) {
        const int j = fdiv(idx, KB), c = idx - j * KB;
        A[c * N + j] = v;
    });
    __syncthreads();
    float2* R = fft<false>(A, B, KB, N, pN, tw);
    float2* O = R == A ? B : A;
    for (int idx = threadIdx.x; idx < N * KB; idx += blockDim.x) {
        const int kj = fdiv(idx, KB), c = idx - kj * KB;
        if (c >= kc) continue;
        const size_t q = (size_t)kj * H + k0 + c;
        const size_t pq = (size_t)plane * N * H + q;
        const float2 v = (mode & 16) ? cadd(R[c * N + kj], yh[pq]) : R[c * N + kj];
        if (mode & 32) {
            yh[pq] = cscale((mode & 3) == 1 && Gt ? cmul(v, Gt[q]) : v, cs);
            continue;
        }
        if (mode & 4) vsave[pq] = v;
        if (mode & 8) {
            const float2 fv = vsave[pq];
            Qp[pq] += (double)v.x * fv.x + (double)v.y * fv.y;
        }
        const int mul = mode & 3;
        R[c * N + kj] = mul == 0 ? cscale(v, cs * Ct[q]) : cmul(v, mul == 1 ? Gt[q] : cconj(Gt[q]));
    }
    if (mode & 32) return;   // block-uniform: Y_h stored, no inverse
    __syncthreads();
    const float2* Z = fft<true>(R, O, KB, N, pN, tw);
    for (int idx = threadIdx.x; idx < N * KB; idx += blockDim.x) {
        const int j = fdiv(idx, KB), c = idx - j * KB;
        if (c < kc) dp[(size_t)j * H + c] = Z[c * N + j];
    }
}

// line update (aniso, iterations 1..K-1) for T lines: s = D x + clip(s_old), w = phi(s),
// v = H^T y + rho D^T w -> half spectrum.  s_old / s_new must not alias (halo line of s_old).
__global__ __launch_bounds__(256) void line_upd_kernel(const float* __restrict__ x, const float* __restrict__ s_old,
                                                       float* __restrict__ s_new, const float* __restrict__ hty,
                                                       float2* __restrict__ spec, const float2* __restrict__ twM,
                                                       FPlan pM, int N, int Tg, const float* __restrict__ prm, int first) {
    const float tau = prm[0]; const float rho = prm[1];   // device-resident scalars (setup_kernel)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int M = pM.n, H = M / 2 + 1;
    const size_t MN = (size_t)M * N;
    float2* A = reinterpret_cast<float2*>(smem_raw);
    float2* B = A + (size_t)((Tg + 1) / 2) * M;   // P = ceil(Tg / 2) paired transforms
    float* W0 = reinterpret_cast<float*>(B + (size_t)((Tg + 1) / 2) * M);   // Tg+1 lines
    float* W1 = W0 + (size_t)(Tg + 1) * M;                       // Tg lines
    const XBlk xb = xcd_block();   // XCD-aware block order (admm_kernels.hip): neighbours share L2 lines
    const int plane = xb.y, j0 = xb.x * Tg;
    const int T = min(Tg, N - j0);   // the last block of a plane may be ragged (gen_nb)
    const float* xp = x + (size_t)plane * MN;
    const float* so = s_old + (size_t)plane * 2 * MN;
    float* sn = s_new + (size_t)plane * 2 * MN;
    struct UpdIn {
        float xc, xu, xl, a0, a1;
    };
    batched<kU>((T + 1) * M, [&](int idx) {
        const int t = fdiv(idx, M), i = idx - t * M;
        const int jj = wrap(j0 + t, N), jp = wrap(jj - 1, N);
        const size_t o = (size_t)jj * M + i;
        UpdIn r;
        r.xc = xp[o];
        r.xu = xp[(size_t)jp * M + i];
        r.xl = t < T ? xp[(size_t)jj * M + wrap(i - 1, M)] : 0.0f;
        r.a0 = first ? 0.0f : so[o];
        r.a1 = (first || t >= T) ? 0.0f : so[MN + o];
        return r;
    }, [&](int idx, const UpdIn& r) {
        const int t = fdiv(idx, M), i = idx - t * M;
        const size_t o = (size_t)wrap(j0 + t, N) * M + i;
        const float s0 = r.xc - r.xu + (first ? 0.0f : clip(r.a0, tau));
        W0[idx] = phi(s0, tau);
        if (t < T) {
            const float s1 = r.xc - r.xl + (first ? 0.0f : clip(r.a1, tau));
            W1[idx] = phi(s1, tau);
            sn[o] = s0;
            sn[MN + o] = s1;
        }
    });
    __syncthreads();
    // hty NULL: H^T y enters spectrally (column_kernel mode 16), v = rho D^T w here
    const float* hp = hty ? hty + (size_t)plane * MN + (size_t)j0 * M : nullptr;
    batched<kU>(T * M, [&](int idx) { return hp ? hp[idx] : 0.0f; }, [&](int idx, float hv) {
        const int t = fdiv(idx, M), i = idx - t * M;
        const float dtw = (W0[idx] - W0[idx + M]) + (W1[idx] - W1[t * M + wrap(i + 1, M)]);
        pack_real(A, t, i, M, fmaf(rho, dtw, hv));
    });
    pad_odd(A, T, M);
    const float2* tw = stage_tw(smem_raw, (size_t)16 * ((Tg + 1) / 2) * M + (size_t)4 * (2 * Tg + 1) * M, twM, M);
    __syncthreads();
    const float2* R = fft<false>(A, B, (T + 1) / 2, M, pM, tw);
    store_real_spectra(R, spec + ((size_t)plane * N + j0) * H, T, M);
}

// isotropic step A (grid (N / T, plane groups)): s = D x + (1 - f_old) s_old (s_in -> s, in place unless
// a trajectory is recorded), and the
// group's partial sum of s^2 over planes and both channels per pixel (ops.jl:6)
__global__ __launch_bounds__(256) void iso_a_kernel(const float* __restrict__ x, const float* s_in, float* s,
                                                    const float* __restrict__ fmap, float* __restrict__ part, int M,
                                                    int N, int planes, int G, int Tg, int first) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float* acc = reinterpret_cast<float*>(smem_raw);
    const size_t MN = (size_t)M * N;
    const int j0 = blockIdx.x * Tg, grp = blockIdx.y;
    const int T = min(Tg, N - j0);   // the last block may be ragged (gen_nb)
    for (int idx = threadIdx.x; idx < T * M; idx += blockDim.x) acc[idx] = 0.0f;
    const int p_end = min(planes, (grp + 1) * G);
    for (int plane = grp * G; plane < p_end; ++plane) {
        const float* xp = x + (size_t)plane * MN;
        float* sp = s + (size_t)plane * 2 * MN;
        const float* si = s_in + (size_t)plane * 2 * MN;   // s_in may alias s (same element read first)
        struct IsoIn {
            float f, xc, xu, xl, a0, a1;
        };
        batched<kU>(T * M, [&](int idx) {
            const int t = fdiv(idx, M), i = idx - t * M;
            const int jj = j0 + t, jp = wrap(jj - 1, N);
            const size_t o = (size_t)jj * M + i;
            IsoIn r;
            r.f = first ? 0.0f : fmap[o];
            r.xc = xp[o];
            r.xu = xp[(size_t)jp * M + i];
            r.xl = xp[(size_t)jj * M + wrap(i - 1, M)];
            r.a0 = first ? 0.0f : si[o];
            r.a1 = first ? 0.0f : si[MN + o];
            return r;
        }, [&](int idx, const IsoIn& r) {
            const int t = fdiv(idx, M), i = idx - t * M;
            const size_t o = (size_t)(j0 + t) * M + i;
            const float s0 = (r.xc - r.xu) + (r.a0 - r.f * r.a0);
            const float s1 = (r.xc - r.xl) + (r.a1 - r.f * r.a1);
            sp[o] = s0;
            sp[MN + o] = s1;
            acc[idx] += s0 * s0 + s1 * s1;   // each idx is owned by one thread
        });
    }
    float* pp = part + (size_t)grp * MN + (size_t)j0 * M;
    for (int idx = threadIdx.x; idx < T * M; idx += blockDim.x) pp[idx] = acc[idx];
}

// isotropic step B: w = (2f - 1) s, v = H^T y + rho D^T w -> half spectrum
__global__ __launch_bounds__(256) void iso_b_kernel(const float* __restrict__ s, const float* __restrict__ fmap,
                                                    const float* __restrict__ hty, float2* __restrict__ spec,
                                                    const float2* __restrict__ twM, FPlan pM, int N, int Tg,
                                                    const float* __restrict__ prm) {
    const float rho = prm[1];   // device-resident scalars (setup_kernel)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int M = pM.n, H = M / 2 + 1;
    const size_t MN = (size_t)M * N;
    float2* A = reinterpret_cast<float2*>(smem_raw);
    float2* B = A + (size_t)((Tg + 1) / 2) * M;   // P = ceil(Tg / 2) paired transforms
    float* W0 = reinterpret_cast<float*>(B + (size_t)((Tg + 1) / 2) * M);
    float* W1 = W0 + (size_t)(Tg + 1) * M;
    const XBlk xb = xcd_block();   // XCD-aware block order (admm_kernels.hip): neighbours share L2 lines
    const int plane = xb.y, j0 = xb.x * Tg;
    const int T = min(Tg, N - j0);   // the last block of a plane may be ragged (gen_nb)
    const float* sp = s + (size_t)plane * 2 * MN;
    batched<kU>((T + 1) * M, [&](int idx) {
        const int t = fdiv(idx, M), i = idx - t * M;
        const size_t o = (size_t)wrap(j0 + t, N) * M + i;
        return make_float3(fmap[o], sp[o], t < T ? sp[MN + o] : 0.0f);
    }, [&](int idx, float3 r) {
        const int t = fdiv(idx, M);
        W0[idx] = r.x * r.y - (r.y - r.x * r.y);
        if (t < T) W1[idx] = r.x * r.z - (r.z - r.x * r.z);
    });
    __syncthreads();
    // hty NULL: H^T y enters spectrally (column_kernel mode 16), v = rho D^T w here
    const float* hp = hty ? hty + (size_t)plane * MN + (size_t)j0 * M : nullptr;
    batched<kU>(T * M, [&](int idx) { return hp ? hp[idx] : 0.0f; }, [&](int idx, float hv) {
        const int t = fdiv(idx, M), i = idx - t * M;
        const float dtw = (W0[idx] - W0[idx + M]) + (W1[idx] - W1[t * M + wrap(i + 1, M)]);
        pack_real(A, t, i, M, fmaf(rho, dtw, hv));
    });
    pad_odd(A, T, M);
    const float2* tw = stage_tw(smem_raw, (size_t)16 * ((Tg + 1) / 2) * M + (size_t)4 * (2 * Tg + 1) * M, twM, M);
    __syncthreads();
    const float2* R = fft<false>(A, B, (T + 1) / 2, M, pM, tw);
    store_real_spectra(R, spec + ((size_t)plane * N + j0) * H, T, M);
}

}  // namespace gen
}  // namespace admm
