// fft_smooth.hpp -- compile-time mixed-radix FFTs for the smooth-length kernels (admm_smooth.hip).
//
// The reference transforms any M x N (FFTW / CUFFT plans, /root/reference/src/ops/ops.jl:26,35-36,86 and
// :108,117-118,168).  admm_generic.hip covers every length with runtime plans; this header gives lengths
// whose prime factors are all <= 31 a plan fixed at compile time:
//   * a transform of LEN points is P <= 4 Stockham passes of radix <= MAXR (make_splan: fewest passes,
//     then the smallest largest radix; radix <= 32: 250 = 25 x 10, 480 = 24 x 20, 640 = 32 x 20;
//     <= 16: 250 = 10 x 5 x 5, 640 = 16 x 8 x 5);
//   * each radix-R butterfly runs in registers: R in {2, 4, 8, 16} as in fft_reg.hpp, odd primes by the
//     symmetric direct form, composite R as A x (R/A) Cooley-Tukey with compile-time twiddles;
//   * pass p maps src[j + r LEN/R] -> dst[(j / Ns) Ns R + j % Ns + r Ns] after the twiddle
//     W_{Ns R}^{r (j % Ns)}, Ns = R_0 ... R_{p-1} (a compile-time constant, so % and / are multiplies).
// Transforms are unnormalised; the forward kernel is exp(-2 pi i n k / LEN).
#pragma once
#include <hip/hip_runtime.h>

#include "fft_reg.hpp"

namespace admm {
namespace sm {

// ---- compile-time trigonometry (twiddles of the in-register DFTs) ----------------------------------
constexpr double kPi = 3.14159265358979323846264338327950288;
// cos / sin of 2 pi e / n by Taylor series on the reduced angle (|x| <= pi: 30 terms are exact in double)
constexpr double taylor_cos(double x) {
    double term = 1.0, sum = 1.0;
    for (int i = 1; i < 30; ++i) {
        term *= -x * x / ((2.0 * i - 1.0) * (2.0 * i));
        sum += term;
    }
    return sum;
}
constexpr double taylor_sin(double x) {
    double term = x, sum = x;
    for (int i = 1; i < 30; ++i) {
        term *= -x * x / ((2.0 * i) * (2.0 * i + 1.0));
        sum += term;
    }
    return sum;
}
constexpr double reduce2pi(long long e, long long n) {
    e %= n;
    if (e < 0) e += n;
    if (2 * e > n) e -= n;   // angle in (-pi, pi]
    return 2.0 * kPi * (double)e / (double)n;
}
constexpr double cos2pi(long long e, long long n) { return taylor_cos(reduce2pi(e, n)); }
constexpr double sin2pi(long long e, long long n) { return taylor_sin(reduce2pi(e, n)); }

template <int R>
struct TrigT {
    float c[R > 0 ? R : 1];
    float s[R > 0 ? R : 1];
};
template <int R>
constexpr TrigT<R> make_trig() {
    TrigT<R> t{};
    for (int e = 0; e < R; ++e) {
        t.c[e] = (float)cos2pi(e, R);
        t.s[e] = (float)sin2pi(e, R);
    }
    return t;
}
template <int R>
constexpr TrigT<R> kTrig = make_trig<R>();

constexpr bool is_prime(int n) {
    if (n < 2) return false;
    for (int d = 2; d * d <= n; ++d)
        if (n % d == 0) return false;
    return true;
}
// largest prime factor of n (1 for n = 1)
constexpr int max_prime(int n) {
    int m = 1;
    for (int d = 2; d <= n; ++d)
        while (n % d == 0) {
            m = d;
            n /= d;
        }
    return m;
}
// lengths this header plans: every prime factor <= 31
constexpr bool plannable(int n) { return n >= 2 && max_prime(n) <= 31; }

// v * W_R^e (forward W_R = exp(-2 pi i / R); inverse: conjugate).  e is a compile-time constant once the
// caller's loops are unrolled, so the quarter-turn cases fold away.
template <int R, bool INV>
__device__ __forceinline__ float2 twc(float2 v, int e) {
    e %= R;
    if (e == 0) return v;
    if (4 * e == R) return rot<INV>(v);
    if (2 * e == R) return make_float2(-v.x, -v.y);
    if (4 * e == 3 * R) return rot<!INV>(v);
    const float c = kTrig<R>.c[e];
    const float s = INV ? kTrig<R>.s[e] : -kTrig<R>.s[e];
    return make_float2(fmaf(v.x, c, -v.y * s), fmaf(v.x, s, v.y * c));
}

// odd prime R, symmetric direct form: t_m = v_m + v_{R-m}, d_m = v_m - v_{R-m};
// X_k = v_0 + sum cos(2 pi m k / R) t_m -/+ i sum sin(2 pi m k / R) d_m
template <int R, bool INV>
__device__ __forceinline__ void dft_odd(float2 (&v)[R]) {
    constexpr int H = (R - 1) / 2;
    float2 t[H + 1], d[H + 1];
#pragma unroll
    for (int m = 1; m <= H; ++m) {
        t[m] = cadd(v[m], v[R - m]);
        d[m] = csub(v[m], v[R - m]);
    }
    float2 x0 = v[0];
#pragma unroll
    for (int m = 1; m <= H; ++m) x0 = cadd(x0, t[m]);
#pragma unroll
    for (int k = 1; k <= H; ++k) {
        float2 a = v[0], b = make_float2(0.f, 0.f);
#pragma unroll
        for (int m = 1; m <= H; ++m) {
            const float c = kTrig<R>.c[(m * k) % R], s = kTrig<R>.s[(m * k) % R];
            a.x = fmaf(c, t[m].x, a.x);
            a.y = fmaf(c, t[m].y, a.y);
            b.x = fmaf(s, d[m].x, b.x);
            b.y = fmaf(s, d[m].y, b.y);
        }
        // forward: X_k = a - i b, X_{R-k} = a + i b (inverse: the other way round)
        const float2 mib = make_float2(b.y, -b.x);
        v[k] = INV ? csub(a, mib) : cadd(a, mib);
        v[R - k] = INV ? cadd(a, mib) : csub(a, mib);
    }
    v[0] = x0;
}

// first factor of a composite radix: a power of two when it has one (cheap inner DFTs), else its
// smallest prime
constexpr int split_a(int R) {
    if (R % 16 == 0 && R > 16) return 16;
    if (R % 8 == 0 && R > 8) return 8;
    if (R % 4 == 0 && R > 4) return 4;
    if (R % 2 == 0 && R > 2) return 2;
    for (int d = 3; d < R; d += 2)
        if (R % d == 0) return d;
    return R;
}

// in-register DFT of R points
template <int R, bool INV>
__device__ __forceinline__ void dftR(float2 (&v)[R]) {
    if constexpr (R == 1) {
    } else if constexpr (R == 2 || R == 4 || R == 8 || R == 16) {
        dft<R, INV>(v);
    } else if constexpr (is_prime(R)) {
        dft_odd<R, INV>(v);
    } else {
        // n = B n1 + n2, k = k1 + A k2:  X = DFT_B over n2 of ( W_R^{n2 k1} DFT_A over n1 )
        constexpr int A = split_a(R), B = R / A;
        float2 y[A][B];
#pragma unroll
        for (int n2 = 0; n2 < B; ++n2) {
            float2 u[A];
#pragma unroll
            for (int n1 = 0; n1 < A; ++n1) u[n1] = v[B * n1 + n2];
            dftR<A, INV>(u);
#pragma unroll
            for (int k1 = 0; k1 < A; ++k1) y[k1][n2] = twc<R, INV>(u[k1], n2 * k1);
        }
#pragma unroll
        for (int k1 = 0; k1 < A; ++k1) {
            float2 w[B];
#pragma unroll
            for (int n2 = 0; n2 < B; ++n2) w[n2] = y[k1][n2];
            dftR<B, INV>(w);
#pragma unroll
            for (int k2 = 0; k2 < B; ++k2) v[k1 + A * k2] = w[k2];
        }
    }
}

// ---- plans -------------------------------------------------------------------------------------------
constexpr int kMaxRadix = 32;   // largest in-register DFT
struct SPlan {
    int P;
    int r[4];
};
constexpr int imax(int a, int b) { return a > b ? a : b; }
constexpr int imin(int a, int b) { return a < b ? a : b; }
// the best plan of n into exactly `passes` radices <= maxr (smallest largest radix; radices in
// non-increasing order); P = 0 if there is none
constexpr SPlan plan_exact(int n, int passes, int maxr) {
    SPlan best{0, {1, 1, 1, 1}};
    if (passes == 1) {
        if (n >= 2 && n <= maxr) best = SPlan{1, {n, 1, 1, 1}};
        return best;
    }
    int best_max = 1 << 30;
    for (int a = 2; a <= maxr; ++a) {
        if (n % a) continue;
        const SPlan sub = plan_exact(n / a, passes - 1, maxr);
        if (!sub.P || sub.r[0] > a) continue;   // keep radices non-increasing (one canonical order)
        const int mx = a;
        if (mx < best_max) {
            best_max = mx;
            best = SPlan{passes, {a, sub.r[0], sub.r[1], sub.r[2]}};
        }
    }
    return best;
}
// ASC: radices in increasing order (the first pass has the most butterflies and the fewest registers per
// butterfly: the line kernels' choice); otherwise decreasing (the column kernel's)
constexpr SPlan make_splan(int n, bool asc, int maxr) {
    for (int p = 1; p <= 4; ++p) {
        SPlan s = plan_exact(n, p, maxr);
        if (s.P) {
            if (asc)
                for (int a = 0, b = s.P - 1; a < b; ++a, --b) {
                    const int t = s.r[a];
                    s.r[a] = s.r[b];
                    s.r[b] = t;
                }
            return s;
        }
    }
    return SPlan{0, {1, 1, 1, 1}};
}
// MAXR: radix cap (more passes, fewer live registers per butterfly when smaller)
template <int LEN, bool ASC = false, int MAXR = kMaxRadix>
struct SP {
    static constexpr SPlan pl = make_splan(LEN, ASC, MAXR);
    static constexpr int P = pl.P;
    static_assert(P >= 1, "length has no plan (a prime factor > 31, or > 32^4)");
    // radix of pass p (REV: the plan run backwards) and the span Ns before it
    template <bool REV>
    static constexpr int radix(int p) { return pl.r[REV ? P - 1 - p : p]; }
    template <bool REV>
    static constexpr int ns(int p) {
        int s = 1;
        for (int q = 0; q < p; ++q) s *= radix<REV>(q);
        return s;
    }
    // most butterflies of any pass of one transform
    static constexpr int max_q() {
        int m = 0;
        for (int q = 0; q < P; ++q) m = imax(m, LEN / pl.r[q]);
        return m;
    }
};

// ---- one Stockham pass over `cnt` transforms, butterflies dealt over the block's NT threads ----------
// Butterfly index idx -> (transform f, butterfly j): FMAJ: f = idx / Q (a transform's butterflies are
// consecutive threads: line transforms); else f = idx % CNTMAX (consecutive threads take consecutive
// transforms: column blocks, coalesced over the columns).  All of a thread's inputs are loaded before any
// output is stored; INPLACE puts a block barrier between the two (src and dst may then be the same LDS).
// tw: LEN-entry table exp(-2 pi i t / LEN).
template <int LEN, int R, int NS, bool INV, int NT, int CNTMAX, bool FMAJ, bool INPLACE, class Load, class Store>
__device__ __forceinline__ void spass(int cnt, const float2* __restrict__ tw, Load&& ld, Store&& st) {
    constexpr int Q = LEN / R;
    constexpr int NR = (CNTMAX * Q + NT - 1) / NT;
    const int total = cnt * Q;
    float2 v[NR][R];
#pragma unroll
    for (int u = 0; u < NR; ++u) {
        const int idx = (int)threadIdx.x + u * NT;
        if (idx < total) {
            const int f = FMAJ ? idx / Q : idx % CNTMAX;
            const int j = FMAJ ? idx - f * Q : idx / CNTMAX;
#pragma unroll
            for (int r = 0; r < R; ++r) v[u][r] = ld(f, j + r * Q);
        }
    }
    if constexpr (INPLACE) __syncthreads();
#pragma unroll
    for (int u = 0; u < NR; ++u) {
        const int idx = (int)threadIdx.x + u * NT;
        if (idx < total) {
            const int f = FMAJ ? idx / Q : idx % CNTMAX;
            const int j = FMAJ ? idx - f * Q : idx / CNTMAX;
            const int k = j % NS;
            if constexpr (NS > 1) {
                constexpr int step = LEN / (NS * R);
#pragma unroll
                for (int r = 1; r < R; ++r) {
                    float2 w = tw[r * k * step];
                    if (INV) w.y = -w.y;
                    v[u][r] = cmul(v[u][r], w);
                }
            }
            dftR<R, INV>(v[u]);
            const int o = (j - k) * R + k;
#pragma unroll
            for (int r = 0; r < R; ++r) st(f, o + r * NS, v[u][r]);
        }
    }
}

// pass p of the plan of LEN (REV: reversed plan; ASC: the increasing-radix plan)
template <int LEN, int p, bool REV, bool INV, int NT, int CNTMAX, bool FMAJ, bool INPLACE, bool ASC = false,
          int MAXR = kMaxRadix, class Load, class Store>
__device__ __forceinline__ void plan_spass(int cnt, const float2* __restrict__ tw, Load&& ld, Store&& st) {
    using S = SP<LEN, ASC, MAXR>;
    spass<LEN, S::template radix<REV>(p), S::template ns<REV>(p), INV, NT, CNTMAX, FMAJ, INPLACE>(cnt, tw, ld, st);
}

// LDS accessor: transform f at base + f * FS, point n
template <int FS>
struct Lds {
    float2* base;
    __device__ __forceinline__ float2 operator()(int f, int n) const { return base[f * FS + n]; }
    __device__ __forceinline__ void operator()(int f, int n, float2 v) const { base[f * FS + n] = v; }
};

// A whole plan, in place in one LDS buffer between the first pass (reads through ld) and the last
// (writes through st).  Barriers between passes; the caller places the ones before and after.
// IN0: ld reads the buffer itself (the first pass is then in place); INL: st writes the buffer.
template <int LEN, bool INV, int NT, int CNTMAX, bool FMAJ, int FS, bool IN0, bool INL, bool ASC = true,
          int MAXR = kMaxRadix, class Load, class Store>
__device__ __forceinline__ void splan(int cnt, const float2* __restrict__ tw, float2* buf, Load&& ld, Store&& st) {
    constexpr int P = SP<LEN, ASC, MAXR>::P;
    const Lds<FS> b{buf};
    if constexpr (P == 1) {
        plan_spass<LEN, 0, false, INV, NT, CNTMAX, FMAJ, IN0 && INL, ASC, MAXR>(cnt, tw, ld, st);
    } else {
        plan_spass<LEN, 0, false, INV, NT, CNTMAX, FMAJ, IN0, ASC, MAXR>(cnt, tw, ld, b);
        __syncthreads();
        if constexpr (P >= 3) {
            plan_spass<LEN, 1, false, INV, NT, CNTMAX, FMAJ, true, ASC, MAXR>(cnt, tw, b, b);
            __syncthreads();
        }
        if constexpr (P >= 4) {
            plan_spass<LEN, 2, false, INV, NT, CNTMAX, FMAJ, true, ASC, MAXR>(cnt, tw, b, b);
            __syncthreads();
        }
        plan_spass<LEN, P - 1, false, INV, NT, CNTMAX, FMAJ, INL, ASC, MAXR>(cnt, tw, b, st);
    }
}

}  // namespace sm
}  // namespace admm
