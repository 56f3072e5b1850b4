// fft_lds.hpp -- block-cooperative Stockham FFTs on LDS-resident lines (gfx950).
//
// The ADMM x-update (reference /root/reference/src/ops/ops.jl:86 / :168) is a 2-D rFFT ->
// spectral scale -> irFFT.  This build splits it into 1-D transforms along dim1 (contiguous
// lines, real <-> half-length complex) and dim2 (strided columns, complex), each executed by a
// whole workgroup on a batch of lines staged in LDS.  Everything here is fp32 with fp64-built
// twiddle tables (a table entry tw[t] = exp(-2*pi*i*t/TWLEN)).
//
// Stockham autosort (Govindaraju et al. / Lloyd-Govindaraju-Smith formulation): pass with
// span Ns and radix R maps src[j + r*LEN/R] -> dst[(j/Ns)*Ns*R + j%Ns + r*Ns] after the
// twiddle W_{Ns R}^{r (j%Ns)}; output lands in natural order, ping-ponging two buffers.
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
// multiply by -i (forward transform) or +i (inverse)
template <bool INV>
__device__ __forceinline__ float2 rot(float2 a) {
    return INV ? make_float2(-a.y, a.x) : make_float2(a.y, -a.x);
}

constexpr int ilog2(int n) { return n <= 1 ? 0 : 1 + ilog2(n >> 1); }

template <int R, bool INV>
__device__ __forceinline__ void butterfly(float2 (&v)[R]) {
    if constexpr (R == 2) {
        float2 a = v[0], b = v[1];
        v[0] = cadd(a, b);
        v[1] = csub(a, b);
    } else {  // R == 4
        float2 s02 = cadd(v[0], v[2]), d02 = csub(v[0], v[2]);
        float2 s13 = cadd(v[1], v[3]), d13 = rot<INV>(csub(v[1], v[3]));
        v[0] = cadd(s02, s13);
        v[2] = csub(s02, s13);
        v[1] = cadd(d02, d13);
        v[3] = csub(d02, d13);
    }
}

// One Stockham pass over `count` independent LEN-point transforms stored with stride
// `fstride` (float2 elements); span Ns = 2^LGNS.  Twiddles come from tw[] of length TWMUL*LEN.
template <int LEN, int R, int LGNS, bool INV, int TWMUL>
__device__ __forceinline__ void stockham_pass(const float2* __restrict__ src, float2* __restrict__ dst,
                                              int count, int fstride, const float2* __restrict__ tw) {
    constexpr int Q = LEN / R;
    constexpr int LGR = ilog2(R);
    constexpr int Ns = 1 << LGNS;
    const int total = count * Q;
    for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
        const int f = idx / Q;
        const int j = idx - f * Q;
        const float2* s = src + f * fstride;
        float2* d = dst + f * fstride;
        const int k = j & (Ns - 1);
        float2 v[R];
#pragma unroll
        for (int r = 0; r < R; ++r) v[r] = s[j + r * Q];
        if constexpr (LGNS > 0) {
            constexpr int step = (Q >> LGNS) * TWMUL;  // LEN/(Ns*R) in table units
#pragma unroll
            for (int r = 1; r < R; ++r) {
                float2 w = tw[r * k * step];
                if (INV) w.y = -w.y;
                v[r] = cmul(v[r], w);
            }
        }
        butterfly<R, INV>(v);
        const int o = ((j - k) << LGR) + k;
#pragma unroll
        for (int r = 0; r < R; ++r) d[o + r * Ns] = v[r];
    }
}

template <int LEN, bool INV, int TWMUL, int LGNS>
__device__ __forceinline__ float2* fft_lds_from(float2* src, float2* dst, int count, int fstride,
                                                const float2* tw) {
    constexpr int LG = ilog2(LEN);
    if constexpr (LGNS + 2 <= LG) {
        stockham_pass<LEN, 4, LGNS, INV, TWMUL>(src, dst, count, fstride, tw);
        __syncthreads();
        return fft_lds_from<LEN, INV, TWMUL, LGNS + 2>(dst, src, count, fstride, tw);
    } else if constexpr (LGNS + 1 == LG) {
        stockham_pass<LEN, 2, LGNS, INV, TWMUL>(src, dst, count, fstride, tw);
        __syncthreads();
        return dst;
    } else {
        return src;
    }
}

// `count` LEN-point transforms on buffer a (b is scratch).  Unnormalised both ways.
// Returns the buffer that holds the result.  Must be called by every thread of the block.
template <int LEN, bool INV, int TWMUL>
__device__ __forceinline__ float2* fft_lds(float2* a, float2* b, int count, int fstride, const float2* tw) {
    return fft_lds_from<LEN, INV, TWMUL, 0>(a, b, count, fstride, tw);
}

}  // namespace admm
