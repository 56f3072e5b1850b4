// admm_kernels.hip -- MI355X (gfx950) kernels for the ADMM TV-deconvolution solve.
//
// Replaces the per-iteration CUFFT/cuDNN/broadcast chain of tvd_fft_gpu
// (/root/reference/src/ops/ops.jl:99-178) with two fused passes per iteration:
//
//   COLUMN pass  (ops.jl:168, the dim2 half of rfft/irfft and the C .* scale):
//       spec0[plane][j][k]  --FFT_j--> xC[k][kj] --IFFT_j-->  spec1[plane][j][k]
//   LINE pass    (ops.jl:168-173 + the dim1 half of the transforms):
//       spec1 --irFFT_i--> x --D--> s = Dx + u --prox--> w = z-u --D^T--> v = H^T y + rho D^T w
//       --rFFT_i--> spec0,     s written back (ping-pong) as the only per-pixel ADMM state.
//
// State compression: with s_k = Dx_k + u_{k-1} the reference's z_k = ST(s_k) and
// u_k = s_k - z_k = clip(s_k, -tau, tau), so z_k - u_k and u_k are functions of s_k alone; one
// 2-channel fp32 tensor replaces the reference's Dx, z, u (ops.jl:128-131).
//
// Half-spectrum packing: a line of M reals has M/2+1 bins, of which bin 0 and bin M/2 are real.
// They share slot 0 as (X[0], X[M/2]), so each line's spectrum is exactly M/2 complex
// (1 KiB for M = 256) and the column pass handles slot 0 with the (C[0]+C[M/2])/2,
// (C[0]-C[M/2])/2 mirror form (both rows of C are even in kj).
//
// Real <-> half-length complex: z[m] = x[2m] + i x[2m+1]; Z = FFT_{M/2}(z);
//   X[k] = E[k] + W_M^k O[k], E = (Z[k] + conj Z[L-k])/2, O = (Z[k] - conj Z[L-k])/(2i).
// All transforms are unnormalised; 1/(M N) is folded into C.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fft_lds.hpp"

namespace admm {

constexpr int kThreads = 256;

// ----------------------------------------------------------------------------------------------
// setup: twiddle tables (double-built) and the C spectrum (ops.jl:22-37)
// ----------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void setup_kernel(float2* __restrict__ twM, float2* __restrict__ twN,
                                                         float* __restrict__ Cmat, const float* __restrict__ h,
                                                         int kh, int kw, int M, int N, float rho) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    double2* tM = reinterpret_cast<double2*>(smem_raw);  // exp(-2 pi i t / M)
    double2* tN = tM + M;                                // exp(-2 pi i t / N)
    for (int t = threadIdx.x; t < M; t += blockDim.x) {
        double s, c;
        sincospi(-2.0 * (double)t / (double)M, &s, &c);
        tM[t] = make_double2(c, s);
    }
    for (int t = threadIdx.x; t < N; t += blockDim.x) {
        double s, c;
        sincospi(-2.0 * (double)t / (double)N, &s, &c);
        tN[t] = make_double2(c, s);
    }
    __syncthreads();
    const int gtid = blockIdx.x * blockDim.x + threadIdx.x;
    const int gsz = gridDim.x * blockDim.x;
    if (blockIdx.x == 0) {
        for (int t = threadIdx.x; t < M; t += blockDim.x) twM[t] = make_float2((float)tM[t].x, (float)tM[t].y);
        for (int t = threadIdx.x; t < N; t += blockDim.x) twN[t] = make_float2((float)tN[t].x, (float)tN[t].y);
    }
    const int L = M / 2;
    const int nbins = (L + 1) * N;
    const double inv_mn = 1.0 / ((double)M * (double)N);
    for (int q = gtid; q < nbins; q += gsz) {
        const int k = q / N;   // dim1 frequency 0..L
        const int kj = q - k * N;
        double s2 = 1.0;
        if (kh > 0) {
            double re = 0.0, im = 0.0;
            for (int b = 0; b < kw; ++b) {
                const double2 eb = tN[(b * kj) & (N - 1)];
                double gr = 0.0, gi = 0.0;
                for (int a = 0; a < kh; ++a) {
                    const double w = (double)h[b * kh + a];
                    const double2 ea = tM[(a * k) & (M - 1)];
                    gr += w * ea.x;
                    gi += w * ea.y;
                }
                re += gr * eb.x - gi * eb.y;
                im += gr * eb.y + gi * eb.x;
            }
            s2 = re * re + im * im;
        }
        const double sx = sinpi((double)kj / (double)N), sy = sinpi((double)k / (double)M);
        const double lap = 4.0 * sx * sx + 4.0 * sy * sy;   // |Lx|^2 + |Ly|^2 (ops.jl:35-36)
        Cmat[q] = (float)(inv_mn / (s2 + (double)rho * lap));
    }
}

// ----------------------------------------------------------------------------------------------
// helpers for the line kernels
// ----------------------------------------------------------------------------------------------
// half-spectrum (packed, L slots) -> half-length complex Z, ready for the inverse L-point FFT
template <int L>
__device__ __forceinline__ void unpack_inverse(const float2* __restrict__ X, float2* __restrict__ Z, int nlines,
                                               const float2* __restrict__ tw) {
    for (int idx = threadIdx.x; idx < nlines * L; idx += blockDim.x) {
        const int t = idx / L;
        const int k = idx - t * L;
        const float2* Xl = X + t * L;
        float2 z;
        if (k == 0) {
            const float2 p = Xl[0];  // (X[0], X[M/2]), both real
            z = make_float2(p.x + p.y, p.x - p.y);
        } else {
            const float2 xk = Xl[k];
            const float2 xm = cconj(Xl[L - k]);
            const float2 e = cadd(xk, xm);
            const float2 o = cmul(csub(xk, xm), cconj(tw[k]));  // * W_M^{-k}
            z = make_float2(e.x - o.y, e.y + o.x);               // E + i O
        }
        Z[idx] = z;
    }
}

// half-length complex spectrum Z -> packed half-spectrum of the real line; writes to global
template <int L>
__device__ __forceinline__ void pack_forward_store(const float2* __restrict__ Z, float2* __restrict__ out_plane,
                                                   int j0, int nlines, int N, const float2* __restrict__ tw) {
    for (int idx = threadIdx.x; idx < nlines * L; idx += blockDim.x) {
        const int t = idx / L;
        const int k = idx - t * L;
        const float2* Zl = Z + t * L;
        float2 X;
        if (k == 0) {
            const float2 z0 = Zl[0];
            X = make_float2(z0.x + z0.y, z0.x - z0.y);
        } else {
            const float2 zk = Zl[k];
            const float2 zm = cconj(Zl[L - k]);
            const float2 e = cscale(cadd(zk, zm), 0.5f);
            const float2 d = csub(zk, zm);
            const float2 o = make_float2(0.5f * d.y, -0.5f * d.x);  // d / (2i)
            X = cadd(e, cmul(tw[k], o));
        }
        const int g = (j0 + t) & (N - 1);
        out_plane[(size_t)g * L + k] = X;
    }
}

__device__ __forceinline__ float clipf(float s, float tau) { return fminf(fmaxf(s, -tau), tau); }
// w = z - u for z = ST(s,tau), u = s - z   (ops.jl:9, :171-173)
__device__ __forceinline__ float prox_w(float s, float tau) {
    const float a = fabsf(s);
    return a > tau ? s - copysignf(2.0f * tau, s) : -s;
}

// load `nlines` packed spectrum lines (j0 + t) mod N into LDS
template <int L>
__device__ __forceinline__ void load_lines(const float2* __restrict__ plane, float2* __restrict__ dst, int j0,
                                           int nlines, int N) {
    const float4* src4 = reinterpret_cast<const float4*>(plane);
    float4* d4 = reinterpret_cast<float4*>(dst);
    constexpr int L2 = L / 2;  // float4 per line
    for (int idx = threadIdx.x; idx < nlines * L2; idx += blockDim.x) {
        const int t = idx / L2;
        const int q = idx - t * L2;
        const int g = (j0 + t) & (N - 1);
        d4[idx] = src4[(size_t)g * L2 + q];
    }
}

// ----------------------------------------------------------------------------------------------
// PREP: H^T y (ops.jl:71-81, computed ONCE; the reference recomputes it every iteration) and the
// first iteration's v = H^T y  (z = u = 0)  ->  rFFT along dim1  ->  spec0
// ----------------------------------------------------------------------------------------------
template <int L>
__global__ __launch_bounds__(kThreads) void prep_kernel(const float* __restrict__ y, float* __restrict__ hty,
                                                        float2* __restrict__ spec0, const float* __restrict__ h,
                                                        int kh, int kw, const float2* __restrict__ twM, int N,
                                                        int T) {
    constexpr int M = 2 * L;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float2* tw = reinterpret_cast<float2*>(smem_raw);
    float2* A = tw + M;
    float2* Bb = A + T * L;
    float* hs = reinterpret_cast<float*>(Bb + T * L);
    float* tile = hs + ((kh * kw + 3) & ~3);
    const int plane = blockIdx.y;
    const int j0 = blockIdx.x * T;
    const float* yp = y + (size_t)plane * N * M;
    for (int t = threadIdx.x; t < M; t += blockDim.x) tw[t] = twM[t];
    float* a_f = reinterpret_cast<float*>(A);
    if (kh > 0) {
        const int padd = (kh - 1) / 2, padr = (kw - 1) / 2;
        for (int t = threadIdx.x; t < kh * kw; t += blockDim.x) hs[t] = h[t];
        const int rows = T + kw - 1;
        constexpr int M4 = M / 4;
        for (int idx = threadIdx.x; idx < rows * M4; idx += blockDim.x) {
            const int r = idx / M4;
            const int q = idx - r * M4;
            const int g = (j0 - padr + r) & (N - 1);
            reinterpret_cast<float4*>(tile)[idx] = reinterpret_cast<const float4*>(yp + (size_t)g * M)[q];
        }
        __syncthreads();
        float* hp = hty + (size_t)plane * N * M;
        for (int idx = threadIdx.x; idx < T * M; idx += blockDim.x) {
            const int t = idx / M;
            const int i = idx - t * M;
            float acc = 0.0f;
            for (int b = 0; b < kw; ++b) {
                const float* row = tile + (t + b) * M;
                const float* hb = hs + b * kh;
                for (int a = 0; a < kh; ++a) acc = fmaf(hb[a], row[(i + a - padd) & (M - 1)], acc);
            }
            a_f[idx] = acc;
            hp[(size_t)((j0 + t) & (N - 1)) * M + i] = acc;
        }
    } else {
        constexpr int M4 = M / 4;
        for (int idx = threadIdx.x; idx < T * M4; idx += blockDim.x) {
            const int t = idx / M4;
            const int q = idx - t * M4;
            const int g = (j0 + t) & (N - 1);
            reinterpret_cast<float4*>(a_f)[idx] = reinterpret_cast<const float4*>(yp + (size_t)g * M)[q];
        }
    }
    __syncthreads();
    float2* R = fft_lds<L, false, 2>(A, Bb, T, L, tw);
    pack_forward_store<L>(R, spec0 + (size_t)plane * N * L, j0, T, N, tw);
}

// ----------------------------------------------------------------------------------------------
// COLUMN pass: for KB consecutive slots of one plane, FFT along dim2 (N points), multiply by C,
// inverse FFT along dim2.  The slot-0 pair (X[0], X[M/2]) uses the even-symmetric mirror form.
// ----------------------------------------------------------------------------------------------
template <int NN>
__global__ __launch_bounds__(kThreads) void column_kernel(const float2* __restrict__ spec0, float2* __restrict__ spec1,
                                                          const float* __restrict__ Cmat,
                                                          const float2* __restrict__ twN, int L, int KB) {
    constexpr int FS = NN + 1;  // padded per-transform stride (transposed staging)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float2* tw = reinterpret_cast<float2*>(smem_raw);
    float2* A = tw + NN;
    float2* Bb = A + KB * FS;
    const int plane = blockIdx.y;
    const int k0 = blockIdx.x * KB;
    const float2* src = spec0 + (size_t)plane * NN * L + k0;
    float2* dst = spec1 + (size_t)plane * NN * L + k0;
    for (int t = threadIdx.x; t < NN; t += blockDim.x) tw[t] = twN[t];
    for (int idx = threadIdx.x; idx < KB * NN; idx += blockDim.x) {
        const int j = idx / KB;
        const int kk = idx - j * KB;
        A[kk * FS + j] = src[(size_t)j * L + kk];
    }
    __syncthreads();
    float2* R = fft_lds<NN, false, 1>(A, Bb, KB, FS, tw);
    float2* O = (R == A) ? Bb : A;
    for (int idx = threadIdx.x; idx < KB * NN; idx += blockDim.x) {
        const int kk = idx / NN;
        const int kj = idx - kk * NN;
        const int k = k0 + kk;
        const float2 z = R[kk * FS + kj];
        float2 o;
        if (k == 0) {
            const float c0 = Cmat[kj], cL = Cmat[(size_t)L * NN + kj];
            const float2 zm = cconj(R[kk * FS + ((NN - kj) & (NN - 1))]);
            o = cadd(cscale(z, 0.5f * (c0 + cL)), cscale(zm, 0.5f * (c0 - cL)));
        } else {
            o = cscale(z, Cmat[(size_t)k * NN + kj]);
        }
        O[kk * FS + kj] = o;
    }
    __syncthreads();
    float2* R2 = fft_lds<NN, true, 1>(O, R, KB, FS, tw);
    for (int idx = threadIdx.x; idx < KB * NN; idx += blockDim.x) {
        const int j = idx / KB;
        const int kk = idx - j * KB;
        dst[(size_t)j * L + kk] = R2[kk * FS + j];
    }
}

// ----------------------------------------------------------------------------------------------
// LINE pass (iterations 1..K-1): T output lines + 1 halo line on each side.
// ----------------------------------------------------------------------------------------------
template <int L>
__global__ __launch_bounds__(kThreads) void line_kernel(const float2* __restrict__ spec1, float2* __restrict__ spec0,
                                                        const float* __restrict__ s_old, float* __restrict__ s_new,
                                                        const float* __restrict__ hty,
                                                        const float2* __restrict__ twM, int N, int T, float tau,
                                                        float rho, int s_zero) {
    constexpr int M = 2 * L;
    constexpr int M4 = M / 4;
    const int TH = T + 2;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float2* tw = reinterpret_cast<float2*>(smem_raw);
    float2* A = tw + M;
    float2* Bb = A + TH * L;
    float* W1 = reinterpret_cast<float*>(Bb + TH * L);  // T lines of M
    const int plane = blockIdx.y;
    const int j0 = blockIdx.x * T;
    const size_t MN = (size_t)M * N;
    for (int t = threadIdx.x; t < M; t += blockDim.x) tw[t] = twM[t];
    load_lines<L>(spec1 + (size_t)plane * N * L, A, j0 - 1, TH, N);
    __syncthreads();
    unpack_inverse<L>(A, Bb, TH, tw);
    __syncthreads();
    float2* Xc = fft_lds<L, true, 2>(Bb, A, TH, L, tw);  // x lines j0-1 .. j0+T
    float* X = reinterpret_cast<float*>(Xc);
    float* W0 = reinterpret_cast<float*>(Xc == A ? Bb : A);  // T+1 lines
    const float* so = s_old + (size_t)plane * 2 * MN;
    float* sn = s_new + (size_t)plane * 2 * MN;
    // s = Dx + u_old ; w = z - u   (ops.jl:169-173)
    for (int idx = threadIdx.x; idx < (T + 1) * M4; idx += blockDim.x) {
        const int t = idx / M4;
        const int i = (idx - t * M4) * 4;
        const int g = (j0 + t) & (N - 1);
        const float4 xc = *reinterpret_cast<const float4*>(X + (t + 1) * M + i);
        const float4 xp = *reinterpret_cast<const float4*>(X + t * M + i);
        float4 so0 = make_float4(0.f, 0.f, 0.f, 0.f);
        if (!s_zero) so0 = *reinterpret_cast<const float4*>(so + (size_t)g * M + i);
        float4 s0;
        s0.x = (xc.x - xp.x) + clipf(so0.x, tau);
        s0.y = (xc.y - xp.y) + clipf(so0.y, tau);
        s0.z = (xc.z - xp.z) + clipf(so0.z, tau);
        s0.w = (xc.w - xp.w) + clipf(so0.w, tau);
        float4 w0 = make_float4(prox_w(s0.x, tau), prox_w(s0.y, tau), prox_w(s0.z, tau), prox_w(s0.w, tau));
        *reinterpret_cast<float4*>(W0 + t * M + i) = w0;
        if (t < T) {
            const float xl = X[(t + 1) * M + ((i - 1) & (M - 1))];
            float4 so1 = make_float4(0.f, 0.f, 0.f, 0.f);
            if (!s_zero) so1 = *reinterpret_cast<const float4*>(so + MN + (size_t)g * M + i);
            float4 s1;
            s1.x = (xc.x - xl) + clipf(so1.x, tau);
            s1.y = (xc.y - xc.x) + clipf(so1.y, tau);
            s1.z = (xc.z - xc.y) + clipf(so1.z, tau);
            s1.w = (xc.w - xc.z) + clipf(so1.w, tau);
            float4 w1 = make_float4(prox_w(s1.x, tau), prox_w(s1.y, tau), prox_w(s1.z, tau), prox_w(s1.w, tau));
            *reinterpret_cast<float4*>(W1 + t * M + i) = w1;
            *reinterpret_cast<float4*>(sn + (size_t)g * M + i) = s0;
            *reinterpret_cast<float4*>(sn + MN + (size_t)g * M + i) = s1;
        }
    }
    __syncthreads();
    // v = H^T y + rho * D^T w   (ops.jl:168)
    const float* hp = hty + (size_t)plane * MN;
    for (int idx = threadIdx.x; idx < T * M4; idx += blockDim.x) {
        const int t = idx / M4;
        const int i = (idx - t * M4) * 4;
        const int g = (j0 + t) & (N - 1);
        const float4 a0 = *reinterpret_cast<const float4*>(W0 + t * M + i);
        const float4 a1 = *reinterpret_cast<const float4*>(W0 + (t + 1) * M + i);
        const float4 b0 = *reinterpret_cast<const float4*>(W1 + t * M + i);
        const float bn = W1[t * M + ((i + 4) & (M - 1))];
        const float4 hv = *reinterpret_cast<const float4*>(hp + (size_t)g * M + i);
        float4 v;
        v.x = fmaf(rho, (a0.x - a1.x) + (b0.x - b0.y), hv.x);
        v.y = fmaf(rho, (a0.y - a1.y) + (b0.y - b0.z), hv.y);
        v.z = fmaf(rho, (a0.z - a1.z) + (b0.z - b0.w), hv.z);
        v.w = fmaf(rho, (a0.w - a1.w) + (b0.w - bn), hv.w);
        *reinterpret_cast<float4*>(X + t * M + i) = v;
    }
    __syncthreads();
    float2* Vin = reinterpret_cast<float2*>(X);
    float2* scratch = reinterpret_cast<float2*>(W0);
    float2* R = fft_lds<L, false, 2>(Vin, scratch, T, L, tw);
    pack_forward_store<L>(R, spec0 + (size_t)plane * N * L, j0, T, N, tw);
}

// ----------------------------------------------------------------------------------------------
// FINAL: last iteration's irFFT along dim1 -> x (ops.jl:168, :175)
// ----------------------------------------------------------------------------------------------
template <int L>
__global__ __launch_bounds__(kThreads) void final_kernel(const float2* __restrict__ spec1, float* __restrict__ x,
                                                         const float2* __restrict__ twM, int N, int T) {
    constexpr int M = 2 * L;
    constexpr int M4 = M / 4;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float2* tw = reinterpret_cast<float2*>(smem_raw);
    float2* A = tw + M;
    float2* Bb = A + T * L;
    const int plane = blockIdx.y;
    const int j0 = blockIdx.x * T;
    for (int t = threadIdx.x; t < M; t += blockDim.x) tw[t] = twM[t];
    load_lines<L>(spec1 + (size_t)plane * N * L, A, j0, T, N);
    __syncthreads();
    unpack_inverse<L>(A, Bb, T, tw);
    __syncthreads();
    float* X = reinterpret_cast<float*>(fft_lds<L, true, 2>(Bb, A, T, L, tw));
    float* xp = x + (size_t)plane * N * M;
    for (int idx = threadIdx.x; idx < T * M4; idx += blockDim.x) {
        const int t = idx / M4;
        const int q = idx - t * M4;
        reinterpret_cast<float4*>(xp + (size_t)(j0 + t) * M)[q] = reinterpret_cast<const float4*>(X + t * M)[q];
    }
}

}  // namespace admm
