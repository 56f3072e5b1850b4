// line_quad.hpp -- register-resident dim-1 transforms of a 256-sample real line held by a LANE QUAD
// (the 1024-thread, 4-waves-per-SIMD layout; line_pair.hpp is the 512-thread lane-pair layout).
//
// Measured and NOT used by the product (tools/line_bench.py): 25 inverse + forward round
// trips of 512 planes' lines in registers take 1.17 ms in this layout (89 VGPRs, 4 waves/SIMD) against
// 1.00 ms in the lane-pair layout (256 VGPRs, 2 waves/SIMD).  The FFT phases are VALU-bound already at
// 2 waves/SIMD, and the second cross-lane radix-2 step and per-lane twiddle selects add VALU work.  So
// the 4-waves-per-SIMD fused kernel that needed this layout was not built.  Kept with its unit test
// (tests/test_gpu_devtest.py) as the reference for that measurement.
//
// Lane q = t & 3 of the quad holding line r (t = 4r + q).  With z[n] = x[2n] + i x[2n+1] (n = 0..127):
//   spatial  : lane q register m holds z[4m + q] = (x[8m + 2q], x[8m + 2q + 1])       m = 0..31
//   spectral : lane q register k holds Z-block p(q) = ((q & 1) << 1) | (q >> 1):
//              X[k + 32 p]  (k = 0..31; lane 0 register 0 = packed (X[0], X[128]))
//   forward: 32-point FFT of each lane's samples (Y_q[k] = sum_m z[4m+q] W32^mk), then the radix-4
//            combine Z[k + 32p] = sum_q W128^qk W4^qp Y_q[k] as two radix-2 steps across the quad
//            (lane bit 1, then lane bit 0; lane q ends with block p(q)), then the real-to-complex
//            post-processing X[j] = (Z[j] + conj Z[128-j])/2 + W256^j (Z[j] - conj Z[128-j])/(2i).
//            The mirror 128 - j of register k (1..31) is register 32 - k of lane 3 - q; register 0
//            pairs lanes 2 and 3 (X[32] / X[96]) and is special on lanes 0 (X[0], X[128]) and 1 (X[64]).
//   inverse: the exact reverse.  Unnormalised both ways: inverse(forward(x)) = 256 x, as line_pair.hpp.
// Every register index is a compile-time constant; cross-lane moves are DPP quad_perm (VALU).
#pragma once
#include <hip/hip_runtime.h>

#include "line_pair.hpp"

namespace admm {
namespace quad {

#ifndef QUAD_FENCE
#define QUAD_FENCE 4   // registers between scheduling fences in the cross-lane steps
#endif

// DPP quad_perm selectors: lane ^ 2, lane ^ 1, 3 - lane
constexpr int kX2 = 0x4E;   // [2,3,0,1]
constexpr int kX1 = 0xB1;   // [1,0,3,2]
constexpr int kMir = 0x1B;  // [3,2,1,0]

template <int CTRL>
__device__ __forceinline__ float qmov(float v) {
    __asm__ volatile("" : "+v"(v));
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
template <int CTRL>
__device__ __forceinline__ float2 qmov2(float2 v) {
    __asm__ volatile("" : "+v"(v.x), "+v"(v.y));
    return make_float2(__int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v.x), CTRL, 0xF, 0xF, true)),
                       __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v.y), CTRL, 0xF, 0xF, true)));
}

// per-lane constants of the quad layout
struct Lane {
    int q;          // lane in quad
    bool a, b;      // q = 2a + b
    int p;          // Z block held after the forward combine: a + 2b
    float2 w8p;     // W256^(32 p) = W8^p (forward); the inverse uses its conjugate
};
__device__ __forceinline__ Lane lane_of(int t) {
    Lane L;
    L.q = t & 3;
    L.a = (L.q >> 1) & 1;
    L.b = L.q & 1;
    L.p = (L.a ? 1 : 0) + (L.b ? 2 : 0);
    constexpr float r = 0.707106781186547524f;
    const float cs[4] = {1.0f, r, 0.0f, -r}, sn[4] = {0.0f, -r, -1.0f, -r};
    L.w8p = make_float2(cs[L.p], sn[L.p]);
    return L;
}

// (branch-free: per-lane selects, no EXEC-masked control flow inside the unrolled transforms)
__device__ __forceinline__ float2 sel(bool c, float2 a, float2 b) { return make_float2(c ? a.x : b.x, c ? a.y : b.y); }

// forward combine step 1 (across lane bit 1): a = 0: Y_b + W64^k Y_{b+2};  a = 1: Y_b - W64^k Y_{b+2}
template <int K>
__device__ __forceinline__ void comb1(float2 (&x)[32], const Lane& L) {
    if constexpr (K < 32) {
        const float2 mine = sel(L.a, w256<4 * K, false>(x[K]), x[K]);
        const float2 oth = qmov2<kX2>(mine);
        x[K] = sel(L.a, csub(oth, mine), cadd(mine, oth));
        if constexpr ((K % QUAD_FENCE) == QUAD_FENCE - 1) sched_fence();
        comb1<K + 1>(x, L);
    }
}
// forward combine step 2 (across lane bit 0): b = 0: U0 + T;  b = 1: U0 - T,  T = W128^(k + 32a) U1
template <int K>
__device__ __forceinline__ void comb2(float2 (&x)[32], const Lane& L) {
    if constexpr (K < 32) {
        // W128^(k + 32a) = W256^(2k) (-i)^a, applied by the b = 1 lanes (branch-free selects)
        const float2 tk = w256<2 * K, false>(x[K]);
        const float2 mine = sel(L.b, sel(L.a, make_float2(tk.y, -tk.x), tk), x[K]);
        const float2 oth = qmov2<kX1>(mine);
        x[K] = sel(L.b, csub(oth, mine), cadd(mine, oth));
        if constexpr ((K % QUAD_FENCE) == QUAD_FENCE - 1) sched_fence();
        comb2<K + 1>(x, L);
    }
}
// inverse of comb2: b = 0: U0 = Z_b0 + Z_b1;  b = 1: U1 = (Z_b0 - Z_b1) conj(W128^(k + 32a))
template <int K>
__device__ __forceinline__ void split2(float2 (&x)[32], const Lane& L) {
    if constexpr (K < 32) {
        const float2 mine = x[K];
        const float2 oth = qmov2<kX1>(mine);
        // conj W128^(k + 32a) = conj W256^(2k) i^a on the b = 1 lanes (branch-free selects)
        const float2 d = w256<2 * K, true>(csub(oth, mine));
        x[K] = sel(L.b, sel(L.a, make_float2(-d.y, d.x), d), cadd(mine, oth));
        if constexpr ((K % QUAD_FENCE) == QUAD_FENCE - 1) sched_fence();
        split2<K + 1>(x, L);
    }
}
// inverse of comb1: a = 0: Y_b = A + B;  a = 1: Y_{b+2} = (A - B) conj(W64^k)
template <int K>
__device__ __forceinline__ void split1(float2 (&x)[32], const Lane& L) {
    if constexpr (K < 32) {
        const float2 mine = x[K];
        const float2 oth = qmov2<kX2>(mine);
        x[K] = sel(L.a, w256<4 * K, true>(csub(oth, mine)), cadd(mine, oth));
        if constexpr ((K % QUAD_FENCE) == QUAD_FENCE - 1) sched_fence();
        split1<K + 1>(x, L);
    }
}

// X[j] = E + W256^j O, E = (Z[j] + conj Z[128-j])/2, O = (Z[j] - conj Z[128-j])/(2i), j = k + 32p:
// W256^j = W256^k W8^p.  zq = the mirror value (raw, from the mirror lane).
template <int K>
__device__ __forceinline__ float2 post(float2 zk, float2 zq, const Lane& L) {
    const float2 zm = cconj(zq);
    const float2 e = cscale(cadd(zk, zm), 0.5f);
    const float2 d = csub(zk, zm);
    const float2 o = cmul(w256<K, false>(make_float2(0.5f * d.y, -0.5f * d.x)), L.w8p);
    return cadd(e, o);
}
// Z[j] = E + i O, E = X[j] + conj X[128-j], O = (X[j] - conj X[128-j]) W256^-j
template <int K>
__device__ __forceinline__ float2 pre(float2 xk, float2 xq, const Lane& L) {
    const float2 xm = cconj(xq);
    const float2 e = cadd(xk, xm);
    const float2 o = cmul(w256<K, true>(csub(xk, xm)), cconj(L.w8p));
    return make_float2(e.x - o.y, e.y + o.x);
}

template <int K>
__device__ __forceinline__ void post_pairs(float2 (&x)[32], const Lane& L) {
    if constexpr (K < 16) {
        constexpr int Q = 32 - K;
        const float2 pq = qmov2<kMir>(x[Q]), pk = qmov2<kMir>(x[K]);
        x[K] = post<K>(x[K], pq, L);
        x[Q] = post<Q>(x[Q], pk, L);
        if constexpr ((K % QUAD_FENCE) == QUAD_FENCE - 1) sched_fence();
        post_pairs<K + 1>(x, L);
    }
}
template <int K>
__device__ __forceinline__ void pre_pairs(float2 (&x)[32], const Lane& L) {
    if constexpr (K < 16) {
        constexpr int Q = 32 - K;
        const float2 pq = qmov2<kMir>(x[Q]), pk = qmov2<kMir>(x[K]);
        x[K] = pre<K>(x[K], pq, L);
        x[Q] = pre<Q>(x[Q], pk, L);
        if constexpr ((K % QUAD_FENCE) == QUAD_FENCE - 1) sched_fence();
        pre_pairs<K + 1>(x, L);
    }
}

// register 0: lane 0 packed (X[0], X[128]) from Z[0]; lane 1 X[64] = conj Z[64]; lanes 2 / 3 the mirror
// pair X[32] / X[96] (partner lane ^ 1)
__device__ __forceinline__ float2 post_r0(float2 z0, const Lane& L) {
    const float2 oth = qmov2<kX1>(z0);
    const float2 g = post<0>(z0, oth, L);
    return sel(L.q == 0, make_float2(z0.x + z0.y, z0.x - z0.y), sel(L.q == 1, cconj(z0), g));
}
__device__ __forceinline__ float2 pre_r0(float2 x0, const Lane& L) {
    const float2 oth = qmov2<kX1>(x0);
    const float2 g = pre<0>(x0, oth, L);
    return sel(L.q == 0, make_float2(x0.x + x0.y, x0.x - x0.y), sel(L.q == 1, make_float2(2.0f * x0.x, -2.0f * x0.y), g));
}

// z (spatial) -> packed half spectrum, in place
__device__ __forceinline__ void line_forward(float2 (&S)[32], const Lane& L) {
    fft_reg<32, false>(S);
    comb1<0>(S, L);
    sched_fence();
    comb2<0>(S, L);
    sched_fence();
    const float2 p16 = qmov2<kMir>(S[16]);
    S[16] = post<16>(S[16], p16, L);
    S[0] = post_r0(S[0], L);
    post_pairs<1>(S, L);
}

// packed half spectrum -> z (spatial), in place (unnormalised: 256 x)
__device__ __forceinline__ void line_inverse(float2 (&S)[32], const Lane& L) {
    const float2 p16 = qmov2<kMir>(S[16]);
    S[16] = pre<16>(S[16], p16, L);
    S[0] = pre_r0(S[0], L);
    pre_pairs<1>(S, L);
    sched_fence();
    split2<0>(S, L);
    sched_fence();
    split1<0>(S, L);
    sched_fence();
    fft_reg<32, true>(S);
}

}  // namespace quad
}  // namespace admm
