// line_pair.hpp -- register-resident dim-1 transforms of a 256-sample real line held by a LANE PAIR.
//
// Used by the fused per-plane kernel (plane_kernel.hip): lane 2r ("A", h = 0) and lane 2r+1 ("B",
// h = 1) hold line r.  With the half-length complex signal z[n] = x[2n] + i x[2n+1] (n = 0..127):
//   spatial  : lane A register n holds z[2n]   = (x[4n],   x[4n+1])     n = 0..63
//              lane B register n holds z[2n+1] = (x[4n+2], x[4n+3])
//   spectral : lane A register m holds X[m]    (m = 0..63; register 0 = packed (X[0], X[128]))
//              lane B register m holds X[64+m]
//   forward: 64-point FFT of each lane's samples (even / odd half of z), the radix-2 DIT combine
//            across the pair (Z[k] = E + W128^k O on A, Z[k+64] = E - W128^k O on B), then the
//            real-to-complex post-processing X[k] = (Z[k] + conj Z[128-k])/2 + W256^k (..)/(2i).
//            The mirror of register m is the PARTNER's register 64-m (m = 1..63), so the post-
//            processing runs in place on register pairs (m, 64-m) with two pair swaps each.
//   inverse: the exact reverse.  Unnormalised both ways: inverse(forward(x)) = 256 x, the same
//            convention as the 2-pass kernels (1/(MN) lives in the spectral tables).
// Every register index is a compile-time constant (no scratch); the only cross-lane operation is the
// pair swap, one DPP quad_perm [1,0,3,2] move per dword.
#pragma once
#include <hip/hip_runtime.h>

#include "fft_reg.hpp"

namespace admm {

#include "tw256.inc"

// (Round 5 measured three instruction-count trims here -- FMA lane-pair add / subtract, exchanges pinned on the
// caller's variable, no select for iteration 1's zero s: 12.4k -> 11.6k VALU per wave, yet c2 5 % slower,
// profiles/r05_plane_xv_ab.jsonl.  They live on as tools/variants/plane_xv.patch, not in this source.)

// v * W256^E (forward, W256 = exp(-2 pi i/256)) or v * conj(W256^E) (inverse)
template <int E, bool INV>
__device__ __forceinline__ float2 w256(float2 v) {
    constexpr int e = E & 255;
    if constexpr (e == 0) {
        return v;
    } else if constexpr (e == 64) {
        return rot<INV>(v);
    } else if constexpr (e == 128) {
        return make_float2(-v.x, -v.y);
    } else if constexpr (e == 192) {
        return rot<!INV>(v);
    } else {
        constexpr float c = kC256[e];
        constexpr float s = INV ? kS256[e] : -kS256[e];
        return make_float2(fmaf(v.x, c, -v.y * s), fmaf(v.x, s, v.y * c));
    }
}

// exchange with the partner lane (lane ^ 1) -- DPP quad_perm [1,0,3,2].
// The empty volatile asm pins the swap's input at its place in the source order: without it
// instruction selection hoists all DPP moves of a transform to its start (~100 extra live VGPRs ->
// scratch spills), ignoring the sched_barrier fences that only bind the machine scheduler.
#ifdef ADMM_SWAP_BPERMUTE
__device__ __forceinline__ float swapf(float v) { return __shfl_xor(v, 1); }
__device__ __forceinline__ float2 swap_pair(float2 v) { return make_float2(__shfl_xor(v.x, 1), __shfl_xor(v.y, 1)); }
#else
__device__ __forceinline__ float swapf(float v) {
    __asm__ volatile("" : "+v"(v));
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
}
__device__ __forceinline__ float2 swap_pair(float2 v) {
    __asm__ volatile("" : "+v"(v.x), "+v"(v.y));
    return make_float2(__int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v.x), 0xB1, 0xF, 0xF, true)),
                       __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v.y), 0xB1, 0xF, 0xF, true)));
}
#endif
// swap_pair of a value the caller uses again: the pin acts on the caller's variable itself, so the swap and the
// later uses read the same (pinned) registers -- pinning a by-value copy made the compiler keep the original
// alive beside it (two v_mov per register of every lane-pair combine)
__device__ __forceinline__ float2 swap_pair_keep(float2& v) {
    return swap_pair(v);
}

// ---- in-register N-point FFT (N = 32 or 64), natural order in and out: N = 4 (n1) x N/4 (n2) -----
//   X[k1 + 4 k2] = sum_{n2} W_{N/4}^{n2 k2} W_N^{n2 k1} sum_{n1} x[(N/4) n1 + n2] W4^{n1 k1}
template <int N, bool INV, int N2>
__device__ __forceinline__ void fftN_tw(float2 (&t)[N / 4][4]) {
    constexpr int S = 256 / N;
    t[N2][1] = w256<S * N2 * 1, INV>(t[N2][1]);
    t[N2][2] = w256<S * N2 * 2, INV>(t[N2][2]);
    t[N2][3] = w256<S * N2 * 3, INV>(t[N2][3]);
    if constexpr (N2 + 1 < N / 4) fftN_tw<N, INV, N2 + 1>(t);
}

// The scheduling fences keep the machine scheduler from interleaving the stages: left free it hoists
// work across them and needs ~260 VGPRs (spilling at 2 waves/SIMD); fenced it needs ~160.
__device__ __forceinline__ void sched_fence() { __builtin_amdgcn_sched_barrier(0); }

template <int N, bool INV>
__device__ __forceinline__ void fft_reg(float2 (&x)[N]) {
    constexpr int Q = N / 4;
    float2 t[Q][4];
#pragma unroll
    for (int n2 = 0; n2 < Q; ++n2) {
        t[n2][0] = x[n2]; t[n2][1] = x[Q + n2]; t[n2][2] = x[2 * Q + n2]; t[n2][3] = x[3 * Q + n2];
        dft4<INV>(t[n2][0], t[n2][1], t[n2][2], t[n2][3]);
    }
    sched_fence();
    fftN_tw<N, INV, 1>(t);
    sched_fence();
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {
        float2 u[Q];
#pragma unroll
        for (int n2 = 0; n2 < Q; ++n2) u[n2] = t[n2][k1];
        dft<Q, INV>(u);
#pragma unroll
        for (int k2 = 0; k2 < Q; ++k2) x[k1 + 4 * k2] = u[k2];
        sched_fence();
    }
}

template <bool INV>
__device__ __forceinline__ void fft64_reg(float2 (&x)[64]) { fft_reg<64, INV>(x); }

// fft_reg<64, INV> whose outputs 32..63 go straight to per-lane LDS slots (stg[m * 512] for m < 16,
// stg2[(m - 16) * 512] above) as soon as their radix-16 group is final, instead of staying live:
// the last stage otherwise needs more than 256 VGPRs and the compiler spills them to scratch.
template <bool INV>
__device__ __forceinline__ void fft64_reg_stage(float2 (&x)[64], float2* stg, float2* stg2) {
    constexpr int Q = 16;
    float2 t[Q][4];
#pragma unroll
    for (int n2 = 0; n2 < Q; ++n2) {
        t[n2][0] = x[n2]; t[n2][1] = x[Q + n2]; t[n2][2] = x[2 * Q + n2]; t[n2][3] = x[3 * Q + n2];
        dft4<INV>(t[n2][0], t[n2][1], t[n2][2], t[n2][3]);
    }
    sched_fence();
    fftN_tw<64, INV, 1>(t);
    sched_fence();
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {
        float2 u[Q];
#pragma unroll
        for (int n2 = 0; n2 < Q; ++n2) u[n2] = t[n2][k1];
        dft<Q, INV>(u);
#pragma unroll
        for (int k2 = 0; k2 < Q; ++k2) {
            const int o = k1 + 4 * k2;
            if (o < 32) x[o] = u[k2];
            else if (o < 48) stg[(o - 32) * 512] = u[k2];
            else stg2[(o - 48) * 512] = u[k2];
        }
        sched_fence();
    }
}

// Lane A adds, lane B subtracts its own value from the partner's: one FMA with the lane's sign sg = +1 (A) / -1
// (B), fma(mine, sg, oth) = mine + oth / oth - mine exactly (a single rounding either way, as the add / sub),
// instead of both results and a select per component.
__device__ __forceinline__ float lane_sign(bool hb) { return hb ? -1.0f : 1.0f; }
__device__ __forceinline__ float2 pm_pair(float2 mine, float2 oth, float sg) {
    return sg < 0.0f ? csub(oth, mine) : cadd(mine, oth);
}

// forward DIT combine across the pair: A: Z[k] = E[k] + W128^k O[k], B: Z[k+64] = E[k] - W128^k O[k]
template <int K>
__device__ __forceinline__ void combine_fwd(float2 (&x)[64], bool hb, float sg) {
    if constexpr (K < 64) {
        float2 xk = x[K];
        // K = 32: W256^64 = -i is a swap of the fields, and `hb ? (y, -x) : (x, y)` on a register still in
        // the front end's S array becomes a select of field ADDRESSES -- S[32] then stays in scratch (the PSF
        // kernel: every access to it a scratch load / store).  The pin makes it a select of values.
        if constexpr (2 * K == 64) __asm__ volatile("" : "+v"(xk.x), "+v"(xk.y));
        float2 mine = hb ? w256<2 * K, false>(xk) : xk;
        const float2 oth = swap_pair_keep(mine);
        x[K] = pm_pair(mine, oth, sg);
        if constexpr ((K & 15) == 15) sched_fence();
        combine_fwd<K + 1>(x, hb, sg);
    }
}

// inverse split across the pair: A: E'[k] = Z[k] + Z[k+64], B: O'[k] = (Z[k] - Z[k+64]) W128^-k
template <int K>
__device__ __forceinline__ void split_inv(float2 (&x)[64], bool hb, float sg) {
    if constexpr (K < 64) {
        float2 mine = x[K];
        const float2 oth = swap_pair_keep(mine);
        const float2 d = pm_pair(mine, oth, sg);
        x[K] = hb ? w256<2 * K, true>(d) : d;
        if constexpr ((K & 15) == 15) sched_fence();
        split_inv<K + 1>(x, hb, sg);
    }
}

// X[k] = E + W256^k O with E = (Z[k] + conj Z[128-k])/2, O = (Z[k] - conj Z[128-k])/(2i);
// k = m (A) or 64 + m (B): W256^(64+m) = -i W256^m.  zq = the partner's register 64-m (raw).
template <int M>
__device__ __forceinline__ float2 post_fwd(float2 zk, float2 zq, bool hb) {
    const float2 zm = cconj(zq);
    const float2 e = cscale(cadd(zk, zm), 0.5f);
    const float2 d = csub(zk, zm);
    float2 o = w256<M, false>(make_float2(0.5f * d.y, -0.5f * d.x));
    if (hb) o = rot<false>(o);
    return cadd(e, o);
}

// Z[k] = E + i O with E = X[k] + conj X[128-k], O = (X[k] - conj X[128-k]) W256^-k; W256^-(64+m) = i W256^-m
template <int M>
__device__ __forceinline__ float2 pre_inv(float2 xk, float2 xq, bool hb) {
    const float2 xm = cconj(xq);
    const float2 e = cadd(xk, xm);
    float2 o = w256<M, true>(csub(xk, xm));
    if (hb) o = rot<true>(o);
    return make_float2(e.x - o.y, e.y + o.x);
}

template <int M>
__device__ __forceinline__ void post_fwd_pairs(float2 (&x)[64], bool hb) {
    if constexpr (M < 32) {
        constexpr int Q = 64 - M;
        const float2 pq = swap_pair_keep(x[Q]), pm = swap_pair_keep(x[M]);
        x[M] = post_fwd<M>(x[M], pq, hb);
        x[Q] = post_fwd<Q>(x[Q], pm, hb);
        if constexpr ((M & 7) == 7) sched_fence();
        post_fwd_pairs<M + 1>(x, hb);
    }
}

template <int M>
__device__ __forceinline__ void pre_inv_pairs(float2 (&x)[64], bool hb) {
    if constexpr (M < 32) {
        constexpr int Q = 64 - M;
        const float2 pq = swap_pair(x[Q]), pm = swap_pair(x[M]);
        x[M] = pre_inv<M>(x[M], pq, hb);
        x[Q] = pre_inv<Q>(x[Q], pm, hb);
        if constexpr ((M & 7) == 7) sched_fence();
        pre_inv_pairs<M + 1>(x, hb);
    }
}

// one register of the inverse split (see split_inv)
template <int K>
__device__ __forceinline__ void split_one(float2 (&x)[64], bool hb, float sg) {
    float2 mine = x[K];
    const float2 oth = swap_pair_keep(mine);
    const float2 d = pm_pair(mine, oth, sg);
    x[K] = hb ? w256<2 * K, true>(d) : d;
}

// pre-processing of pair (M, 64-M) fused with the split of both registers: each register is final for
// the 64-point IFFT as soon as its pair is done, which keeps the live set small (pre then split as two
// sweeps needed ~256 VGPRs and spilled; fused it fits with the FFT's own peak)
template <int M>
__device__ __forceinline__ void pre_split_pairs(float2 (&x)[64], bool hb, float sg) {
    if constexpr (M < 32) {
        constexpr int Q = 64 - M;
        const float2 pq = swap_pair_keep(x[Q]), pm = swap_pair_keep(x[M]);
        x[M] = pre_inv<M>(x[M], pq, hb);
        x[Q] = pre_inv<Q>(x[Q], pm, hb);
        split_one<M>(x, hb, sg);
        split_one<Q>(x, hb, sg);
        if constexpr ((M & 3) == 3) sched_fence();
        pre_split_pairs<M + 1>(x, hb, sg);
    }
}

// z (spatial) -> packed half spectrum, in place
__device__ __forceinline__ void line_forward_pair(float2 (&S)[64], bool hb) {
    fft64_reg<false>(S);
    combine_fwd<0>(S, hb, lane_sign(hb));
    sched_fence();
    // k = 0 (A): packed (X[0], X[128]) = (Re Z0 + Im Z0, Re Z0 - Im Z0); k = 64 (B): X[64] = conj Z[64]
    const float2 z0 = S[0];
    S[0] = hb ? cconj(z0) : make_float2(z0.x + z0.y, z0.x - z0.y);
    const float2 p32 = swap_pair(S[32]);
    S[32] = post_fwd<32>(S[32], p32, hb);
    post_fwd_pairs<1>(S, hb);
}

// line_inverse_pair with z registers 32..63 delivered to the LDS staging slots (fft64_reg_stage)
__device__ __forceinline__ void line_inverse_pair_staged(float2 (&S)[64], bool hb, float2* stg, float2* stg2) {
    const float sg = lane_sign(hb);
    const float2 x0 = S[0];
    S[0] = hb ? make_float2(2.f * x0.x, -2.f * x0.y) : make_float2(x0.x + x0.y, x0.x - x0.y);
    split_one<0>(S, hb, sg);
    const float2 p32 = swap_pair(S[32]);
    S[32] = pre_inv<32>(S[32], p32, hb);
    split_one<32>(S, hb, sg);
    pre_split_pairs<1>(S, hb, sg);
    sched_fence();
    fft64_reg_stage<true>(S, stg, stg2);
}

// packed half spectrum -> z (spatial), in place (unnormalised: 256 x)
__device__ __forceinline__ void line_inverse_pair(float2 (&S)[64], bool hb) {
    const float sg = lane_sign(hb);
    const float2 x0 = S[0];
    S[0] = hb ? make_float2(2.f * x0.x, -2.f * x0.y) : make_float2(x0.x + x0.y, x0.x - x0.y);
    split_one<0>(S, hb, sg);
    const float2 p32 = swap_pair(S[32]);
    S[32] = pre_inv<32>(S[32], p32, hb);
    split_one<32>(S, hb, sg);
    pre_split_pairs<1>(S, hb, sg);
    sched_fence();
    fft64_reg<true>(S);
}

}  // namespace admm
