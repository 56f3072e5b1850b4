// fft_reg.hpp -- register-resident radix-2/4/8/16 butterflies and a Stockham pass with pluggable
// load/store, for block-cooperative FFTs of lines staged in LDS (gfx950, wave64).
//
// The ADMM x-update (reference /root/reference/src/ops/ops.jl:86 / :168) is a 2-D rFFT -> spectral
// scale -> irFFT.  This build runs it as 1-D transforms along dim1 (contiguous lines) and dim2
// (strided columns).  Each transform of length LEN is a short Stockham plan of radix-8/16 passes
// (256 = 16x16, 128 = 16x8 ...): a pass loads R points per thread, twiddles, runs an in-register
// R-point DFT and stores them.  Load/store are callables so the first pass can read global memory
// (or compute its input) and the last pass can write global memory (or feed the next stage), which
// removes LDS round trips and barriers.
//
// Stockham autosort: pass with span Ns = 2^LGNS and radix R maps src[j + r*LEN/R] to
// dst[(j/Ns)*Ns*R + j%Ns + r*Ns] after the twiddle W_{Ns R}^{r (j%Ns)}; output is in natural order.
// Transforms are unnormalised; the forward kernel is exp(-2 pi i n k / LEN).
#pragma once
#include <hip/hip_runtime.h>

namespace admm {

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
// multiply by -i (forward) or +i (inverse)
template <bool INV>
__device__ __forceinline__ float2 rot(float2 a) {
    return INV ? make_float2(-a.y, a.x) : make_float2(a.y, -a.x);
}

constexpr int ilog2(int n) { return n <= 1 ? 0 : 1 + ilog2(n >> 1); }

// cos / sin of 2*pi*e/16
constexpr float kC16[16] = {1.0f, 0.923879532511286756f, 0.707106781186547524f, 0.382683432365089772f,
                            0.0f, -0.382683432365089772f, -0.707106781186547524f, -0.923879532511286756f,
                            -1.0f, -0.923879532511286756f, -0.707106781186547524f, -0.382683432365089772f,
                            0.0f, 0.382683432365089772f, 0.707106781186547524f, 0.923879532511286756f};
constexpr float kS16[16] = {0.0f, 0.382683432365089772f, 0.707106781186547524f, 0.923879532511286756f,
                            1.0f, 0.923879532511286756f, 0.707106781186547524f, 0.382683432365089772f,
                            0.0f, -0.382683432365089772f, -0.707106781186547524f, -0.923879532511286756f,
                            -1.0f, -0.923879532511286756f, -0.707106781186547524f, -0.382683432365089772f};

// v * W16^E (forward, W16 = exp(-2 pi i/16)) or v * conj(W16^E) (inverse)
template <int E, bool INV>
__device__ __forceinline__ float2 w16(float2 v) {
    constexpr int e = E & 15;
    if constexpr (e == 0) {
        return v;
    } else if constexpr (e == 4) {
        return rot<INV>(v);
    } else if constexpr (e == 8) {
        return make_float2(-v.x, -v.y);
    } else if constexpr (e == 12) {
        return rot<!INV>(v);
    } else {
        constexpr float c = kC16[e];
        constexpr float s = INV ? kS16[e] : -kS16[e];
        return make_float2(fmaf(v.x, c, -v.y * s), fmaf(v.x, s, v.y * c));
    }
}

template <bool INV>
__device__ __forceinline__ void dft2(float2& a, float2& b) {
    const float2 t = a;
    a = cadd(t, b);
    b = csub(t, b);
}

template <bool INV>
__device__ __forceinline__ void dft4(float2& v0, float2& v1, float2& v2, float2& v3) {
    const float2 s02 = cadd(v0, v2), d02 = csub(v0, v2);
    const float2 s13 = cadd(v1, v3), d13 = rot<INV>(csub(v1, v3));
    v0 = cadd(s02, s13);
    v2 = csub(s02, s13);
    v1 = cadd(d02, d13);
    v3 = csub(d02, d13);
}

template <int R, bool INV>
__device__ __forceinline__ void dft(float2 (&v)[R]) {
    if constexpr (R == 1) {
    } else if constexpr (R == 2) {
        dft2<INV>(v[0], v[1]);
    } else if constexpr (R == 4) {
        dft4<INV>(v[0], v[1], v[2], v[3]);
    } else if constexpr (R == 8) {
        // radix-2 (stride 4) then two radix-4: X[2p] = DFT4(a)[p], X[2p+1] = DFT4(b W8^q)[p]
        float2 a0 = cadd(v[0], v[4]), a1 = cadd(v[1], v[5]), a2 = cadd(v[2], v[6]), a3 = cadd(v[3], v[7]);
        float2 b0 = csub(v[0], v[4]), b1 = csub(v[1], v[5]), b2 = csub(v[2], v[6]), b3 = csub(v[3], v[7]);
        b1 = w16<2, INV>(b1);
        b2 = w16<4, INV>(b2);
        b3 = w16<6, INV>(b3);
        dft4<INV>(a0, a1, a2, a3);
        dft4<INV>(b0, b1, b2, b3);
        v[0] = a0; v[2] = a1; v[4] = a2; v[6] = a3;
        v[1] = b0; v[3] = b1; v[5] = b2; v[7] = b3;
    } else {  // R == 16: 4 x 4 with W16^{q m} between; X[m + 4p]
        float2 a[4][4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            a[q][0] = v[q]; a[q][1] = v[q + 4]; a[q][2] = v[q + 8]; a[q][3] = v[q + 12];
            dft4<INV>(a[q][0], a[q][1], a[q][2], a[q][3]);
        }
        a[1][1] = w16<1, INV>(a[1][1]);
        a[1][2] = w16<2, INV>(a[1][2]);
        a[1][3] = w16<3, INV>(a[1][3]);
        a[2][1] = w16<2, INV>(a[2][1]);
        a[2][2] = w16<4, INV>(a[2][2]);
        a[2][3] = w16<6, INV>(a[2][3]);
        a[3][1] = w16<3, INV>(a[3][1]);
        a[3][2] = w16<6, INV>(a[3][2]);
        a[3][3] = w16<9, INV>(a[3][3]);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            dft4<INV>(a[0][m], a[1][m], a[2][m], a[3][m]);
            v[m] = a[0][m]; v[m + 4] = a[1][m]; v[m + 8] = a[2][m]; v[m + 12] = a[3][m];
        }
    }
}

// ---- radix plans: LEN = R0 * R1 * R2 (pass p runs with Ns = R0*...*R(p-1)) -------------------
template <int LEN>
struct Plan;
template <> struct Plan<2>    { static constexpr int P = 1, R0 = 2,  R1 = 1, R2 = 1; };
template <> struct Plan<4>    { static constexpr int P = 1, R0 = 4,  R1 = 1, R2 = 1; };
template <> struct Plan<8>    { static constexpr int P = 1, R0 = 8,  R1 = 1, R2 = 1; };
template <> struct Plan<16>   { static constexpr int P = 1, R0 = 16, R1 = 1, R2 = 1; };
template <> struct Plan<32>   { static constexpr int P = 2, R0 = 8,  R1 = 4, R2 = 1; };
template <> struct Plan<64>   { static constexpr int P = 2, R0 = 8,  R1 = 8, R2 = 1; };
template <> struct Plan<128>  { static constexpr int P = 2, R0 = 16, R1 = 8, R2 = 1; };
template <> struct Plan<256>  { static constexpr int P = 2, R0 = 16, R1 = 16, R2 = 1; };
template <> struct Plan<512>  { static constexpr int P = 3, R0 = 8,  R1 = 8, R2 = 8; };
template <> struct Plan<1024> { static constexpr int P = 3, R0 = 16, R1 = 8, R2 = 8; };

template <int LEN, int p, bool REV>
constexpr int plan_radix() {
    using PL = Plan<LEN>;
    constexpr int q = REV ? PL::P - 1 - p : p;
    return q == 0 ? PL::R0 : (q == 1 ? PL::R1 : PL::R2);
}
template <int LEN, int p, bool REV>
constexpr int plan_lgns() {
    if constexpr (p == 0) return 0;
    else return plan_lgns<LEN, p - 1, REV>() + ilog2(plan_radix<LEN, p - 1, REV>());
}
template <int LEN, bool REV>
constexpr int plan_max_q() {  // largest number of butterflies per transform over the plan
    using PL = Plan<LEN>;
    int m = LEN / PL::R0;
    if (PL::P > 1 && LEN / PL::R1 > m) m = LEN / PL::R1;
    if (PL::P > 2 && LEN / PL::R2 > m) m = LEN / PL::R2;
    return m;
}

// Twiddle + in-register DFT of one Stockham butterfly whose R inputs are already in v[].
// Outputs go to index out_index(j, r).
template <int LEN, int R, int LGNS, bool INV, int TWMUL>
__device__ __forceinline__ void fly_core(float2 (&v)[R], int j, const float2* __restrict__ tw) {
    constexpr int Q = LEN / R;
    constexpr int Ns = 1 << LGNS;
    if constexpr (LGNS > 0) {
        const int k = j & (Ns - 1);
        constexpr int step = (Q >> LGNS) * TWMUL;   // LEN/(Ns R) in table units
#pragma unroll
        for (int r = 1; r < R; ++r) {
            float2 w = tw[r * k * step];
            if (INV) w.y = -w.y;
            v[r] = cmul(v[r], w);
        }
    }
    dft<R, INV>(v);
}
template <int LEN, int R, int LGNS>
__device__ __forceinline__ int out_base(int j) {
    constexpr int Ns = 1 << LGNS;
    const int k = j & (Ns - 1);
    return ((j - k) << ilog2(R)) + k;
}

// One butterfly of a Stockham pass for transform f, index j (0 <= j < LEN/R).
template <int LEN, int R, int LGNS, bool INV, int TWMUL, class Load, class Store>
__device__ __forceinline__ void fly(int f, int j, const float2* __restrict__ tw, Load&& load, Store&& store) {
    constexpr int Q = LEN / R;
    constexpr int Ns = 1 << LGNS;
    float2 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = load(f, j + r * Q);
    fly_core<LEN, R, LGNS, INV, TWMUL>(v, j, tw);
    const int o = out_base<LEN, R, LGNS>(j);
#pragma unroll
    for (int r = 0; r < R; ++r) store(f, o + r * Ns, v[r]);
}

// Full Stockham pass over `count` transforms, work-shared by the block (grid-stride on threads).
template <int LEN, int R, int LGNS, bool INV, int TWMUL, class Load, class Store>
__device__ __forceinline__ void fpass(int count, const float2* __restrict__ tw, Load&& load, Store&& store) {
    constexpr int Q = LEN / R;
    const int total = count * Q;
    for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
        const int f = idx / Q;
        fly<LEN, R, LGNS, INV, TWMUL>(f, idx - f * Q, tw, load, store);
    }
}

// Plan pass p of transform length LEN (REV = plan reversed).
template <int LEN, int p, bool REV, bool INV, int TWMUL, class Load, class Store>
__device__ __forceinline__ void plan_pass(int count, const float2* __restrict__ tw, Load&& load, Store&& store) {
    fpass<LEN, plan_radix<LEN, p, REV>(), plan_lgns<LEN, p, REV>(), INV, TWMUL>(count, tw, load, store);
}

// LDS accessors (transform f at base + f*fstride)
struct LdsIO {
    float2* base;
    int fstride;
    __device__ __forceinline__ float2 operator()(int f, int n) const { return base[f * fstride + n]; }
    __device__ __forceinline__ void operator()(int f, int n, float2 v) const { base[f * fstride + n] = v; }
};

// Run a whole plan: first pass loads through `load`, last pass stores through `store`; intermediate
// results ping-pong between LDS buffers b0 and b1 (neither may alias load's source while pass 0 runs).
// Barriers are placed between passes; the caller places the ones before and after.
template <int LEN, bool REV, bool INV, int TWMUL, class Load, class Store>
__device__ __forceinline__ void fft_plan(int count, const float2* __restrict__ tw, float2* b0, float2* b1,
                                         int fstride, Load&& load, Store&& store) {
    constexpr int P = Plan<LEN>::P;
    const LdsIO s0{b0, fstride}, s1{b1, fstride};
    if constexpr (P == 1) {
        plan_pass<LEN, 0, REV, INV, TWMUL>(count, tw, load, store);
    } else if constexpr (P == 2) {
        plan_pass<LEN, 0, REV, INV, TWMUL>(count, tw, load, s0);
        __syncthreads();
        plan_pass<LEN, 1, REV, INV, TWMUL>(count, tw, s0, store);
    } else {
        plan_pass<LEN, 0, REV, INV, TWMUL>(count, tw, load, s0);
        __syncthreads();
        plan_pass<LEN, 1, REV, INV, TWMUL>(count, tw, s0, s1);
        __syncthreads();
        plan_pass<LEN, 2, REV, INV, TWMUL>(count, tw, s1, store);
    }
}

}  // namespace admm
