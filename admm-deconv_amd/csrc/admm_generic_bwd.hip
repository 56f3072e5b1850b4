// admm_generic_bwd.hip -- reverse sweep (adjoint) for shapes outside the
// power-of-two kernels: the same recurrences as admm_backward.hip (its header states them;
// tests/kernel_model.py tvd_model_grads restates them) on the runtime-length layout of
// admm_generic.hip (spectrum [plane][line j][bin k], H = M/2 + 1 bins; x / vbar through HBM).
//   step k = K..1:  GEN_COLUMN (x C/(MN), + Q against the forward spectra for h_bar)
//                   GEN_LINE_INV -> vbar_k
//                   aniso: GEN_LINE_ADJ (D vbar, rho/tau partials, Vsum, sbar_{k-1}, D^T sbar -> dim-1 FFT)
//                   iso:   GEN_ISO_ADJ_A (plane groups) -> ISO_ADJ_R -> GEN_ISO_ADJ_B (D^T sbar -> dim-1 FFT)
#include <hip/hip_runtime.h>

namespace admm {
namespace gen {

__device__ __forceinline__ float sgn1(float s) { return s > 0.f ? 1.0f : -1.0f; }

// block sum of two floats in fp64, fixed order; thread 0 writes out[0..1]
__device__ __forceinline__ void block_pair(float a, float b, double* out) {
    __shared__ double red[2 * 16];
    double da = a, db = b;
    for (int off = 32; off > 0; off >>= 1) {
        da += __shfl_down(da, off);
        db += __shfl_down(db, off);
    }
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) {
        red[2 * w] = da;
        red[2 * w + 1] = db;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double sa = 0.0, sb = 0.0;
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
            sa += red[2 * i];
            sb += red[2 * i + 1];
        }
        out[0] = sa;
        out[1] = sb;
    }
}

// D x_k at pixel (i, j) of a plane: k = K from the forward output xK, else s_k - clip(s_{k-1})
__device__ __forceinline__ void dx_at(const float* __restrict__ xK, const float* __restrict__ sk,
                                      const float* __restrict__ sk1, int i, int j, int M, int N, size_t MN, float tau,
                                      float& d0, float& d1) {
    const size_t o = (size_t)j * M + i;
    if (xK) {
        const float xc = xK[o];
        d0 = xc - xK[(size_t)wrap(j - 1, N) * M + i];
        d1 = xc - xK[(size_t)j * M + wrap(i - 1, M)];
    } else {
        d0 = sk[o] - (sk1 ? clip(sk1[o], tau) : 0.0f);
        d1 = sk[MN + o] - (sk1 ? clip(sk1[MN + o], tau) : 0.0f);
    }
}

// Aniso reverse step for T lines of one plane (grid (N / T, planes), 256 threads).
//   vb: vbar_k (spatial, HBM)    sk1: s_{k-1} (null at k = 1)   sk: s_k (null at k = K: xK used)
//   sb_in: sbar_k (null at k = K)   sb_out: sbar_{k-1}   vsum += vbar_k   spec: dim-1 FFT of D^T sbar_{k-1}
//   part: (rho_bar, tau_bar) partial of this block
__global__ __launch_bounds__(256) void line_adj_kernel(const float* __restrict__ vb, const float* __restrict__ sk1,
                                                       const float* __restrict__ sk, const float* __restrict__ xK,
                                                       const float* __restrict__ sb_in, float* __restrict__ sb_out,
                                                       float* __restrict__ vsum, float2* __restrict__ spec,
                                                       double* __restrict__ part, const float2* __restrict__ twM,
                                                       FPlan pM, int N, int T, const float* __restrict__ prm) {
    const float tau = prm[0]; const float rho = prm[1];   // device-resident scalars (setup_kernel / scal_kernel)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int M = pM.n, H = M / 2 + 1;
    const size_t MN = (size_t)M * N;
    float2* A = reinterpret_cast<float2*>(smem_raw);
    float2* B = A + (size_t)((T + 1) / 2) * M;   // P = ceil(T / 2) paired transforms
    float* W0 = reinterpret_cast<float*>(B + (size_t)((T + 1) / 2) * M);   // sbar_{k-1} ch0, T+1 lines
    float* W1 = W0 + (size_t)(T + 1) * M;                       // sbar_{k-1} ch1, T lines
    float* V = reinterpret_cast<float*>(smem_raw);              // vbar lines j0-1 .. j0+T (aliases A, B)
    const XBlk xb = xcd_block();   // XCD-aware block order (admm_kernels.hip): neighbours share L2 lines
    const int plane = xb.y, j0 = xb.x * T;
    const size_t poff = (size_t)plane * 2 * MN;
    const float* vp = vb + (size_t)plane * MN;
    for (int idx = threadIdx.x; idx < (T + 2) * M; idx += blockDim.x) {
        const int t = fdiv(idx, M), i = idx - t * M;
        V[idx] = vp[(size_t)wrap(j0 - 1 + t, N) * M + i];
    }
    __syncthreads();
    const float* xk = (xK && !sk) ? xK + (size_t)plane * MN : nullptr;
    const float* skp = sk ? sk + poff : nullptr;
    const float* s1p = sk1 ? sk1 + poff : nullptr;
    float racc = 0.0f, tacc = 0.0f;
    for (int idx = threadIdx.x; idx < (T + 1) * M; idx += blockDim.x) {
        const int t = fdiv(idx, M), i = idx - t * M;
        const int j = wrap(j0 + t, N);
        const size_t o = (size_t)j * M + i;
        const bool own = t < T;
        const float vc = V[(t + 1) * M + i];
        const float dv0 = vc - V[t * M + i];
        const float dv1 = vc - V[(t + 1) * M + wrap(i - 1, M)];
        const float a0 = s1p ? s1p[o] : 0.0f;
        const float a1 = (s1p && own) ? s1p[MN + o] : 0.0f;
        if (own) {
            float d0, d1;
            dx_at(xk, skp, s1p, i, j, M, N, MN, tau, d0, d1);
            racc -= dv0 * d0 + dv1 * d1;
            vsum[(size_t)plane * MN + o] += vc;
        }
        if (!s1p) continue;   // k = 1: no sbar_0 (block-uniform)
        const float b0 = sb_in ? sb_in[poff + o] : 0.0f;
        const float w0 = rho * dv0;
        const bool m0 = fabsf(a0) > tau;
        const float n0 = m0 ? w0 : b0 - w0;
        W0[idx] = n0;
        if (own) {
            const float b1 = sb_in ? sb_in[poff + MN + o] : 0.0f;
            const float w1 = rho * dv1;
            const bool m1 = fabsf(a1) > tau;
            const float n1 = m1 ? w1 : b1 - w1;
            W1[idx] = n1;
            racc += phi(a0, tau) * dv0 + phi(a1, tau) * dv1;
            tacc += (m0 ? sgn1(a0) * (b0 - 2.0f * w0) : 0.0f) + (m1 ? sgn1(a1) * (b1 - 2.0f * w1) : 0.0f);
            sb_out[poff + o] = n0;
            sb_out[poff + MN + o] = n1;
        }
    }
    block_pair(racc, tacc, part + 2 * ((size_t)plane * gridDim.x + xb.x));
    if (!s1p) return;
    __syncthreads();   // W0/W1 complete; V (aliasing A, B) is dead
    for (int idx = threadIdx.x; idx < T * M; idx += blockDim.x) {
        const int t = fdiv(idx, M), i = idx - t * M;
        const float g = (W0[idx] - W0[idx + M]) + (W1[idx] - W1[t * M + wrap(i + 1, M)]);
        pack_real(A, t, i, M, g);
    }
    pad_odd(A, T, M);
    const float2* tw = stage_tw(smem_raw, (size_t)16 * ((T + 1) / 2) * M + (size_t)4 * (2 * T + 1) * M, twM, M);
    __syncthreads();
    const float2* R = fft<false>(A, B, (T + 1) / 2, M, pM, tw);
    store_real_spectra(R, spec + ((size_t)plane * N + j0) * H, T, M);
}

// Iso reverse step A (grid (N / T, plane groups)): per plane of the group D vbar, rho_bar partial,
// Vsum += vbar, wbar = rho D vbar (stored); per pixel the group's partial
// R = sum s_{k-1} (2 wbar - sbar_k) over its planes and both channels (admm_backward.hip, iso section).
//   nrm1: batch norm of s_{k-1} (null at k = 1)
__global__ __launch_bounds__(256) void iso_adj_a_kernel(const float* __restrict__ vb, const float* __restrict__ sk1,
                                                        const float* __restrict__ sk, const float* __restrict__ xK,
                                                        const float* __restrict__ nrm1, const float* __restrict__ sb_in,
                                                        float* __restrict__ vbar_out, float* __restrict__ vsum,
                                                        float* __restrict__ rpartial, double* __restrict__ part,
                                                        int M, int N, int planes, int G, int T, const float* __restrict__ prm) {
    const float tau = prm[0]; const float rho = prm[1];   // device-resident scalars (setup_kernel / scal_kernel)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float* acc = reinterpret_cast<float*>(smem_raw);
    const size_t MN = (size_t)M * N;
    const int j0 = blockIdx.x * T, grp = blockIdx.y;
    for (int idx = threadIdx.x; idx < T * M; idx += blockDim.x) acc[idx] = 0.0f;
    float racc = 0.0f;
    const int p_end = min(planes, (grp + 1) * G);
    for (int plane = grp * G; plane < p_end; ++plane) {
        const float* vp = vb + (size_t)plane * MN;
        const size_t poff = (size_t)plane * 2 * MN;
        for (int idx = threadIdx.x; idx < T * M; idx += blockDim.x) {
            const int t = fdiv(idx, M), i = idx - t * M;
            const int j = j0 + t;
            const size_t o = (size_t)j * M + i;
            const float vc = vp[o];
            const float dv0 = vc - vp[(size_t)wrap(j - 1, N) * M + i];
            const float dv1 = vc - vp[(size_t)j * M + wrap(i - 1, M)];
            const float f = nrm1 ? max0_nan(1.0f - tau / nrm1[o]) : 0.0f;   // BT factor of s_{k-1}
            const float a0 = sk1 ? sk1[poff + o] : 0.0f, a1 = sk1 ? sk1[poff + MN + o] : 0.0f;
            float d0, d1;   // D x_k = s_k - psi(s_{k-1}) = s_k - (1 - f) s_{k-1}, or from xK at k = K
            if (!sk) {
                const float* xp = xK + (size_t)plane * MN;
                const float xc = xp[o];
                d0 = xc - xp[(size_t)wrap(j - 1, N) * M + i];
                d1 = xc - xp[(size_t)j * M + wrap(i - 1, M)];
            } else {
                d0 = sk[poff + o] - (1.0f - f) * a0;
                d1 = sk[poff + MN + o] - (1.0f - f) * a1;
            }
            racc -= dv0 * d0 + dv1 * d1;
            vsum[(size_t)plane * MN + o] += vc;
            if (sk1) {
                const float b0 = sb_in ? sb_in[poff + o] : 0.0f, b1 = sb_in ? sb_in[poff + MN + o] : 0.0f;
                const float w0 = rho * dv0, w1 = rho * dv1;
                racc += (2.0f * f - 1.0f) * (a0 * dv0 + a1 * dv1);   // phi(s) = (2f - 1) s
                acc[idx] += a0 * (2.0f * w0 - b0) + a1 * (2.0f * w1 - b1);
                vbar_out[(size_t)plane * MN + o] = vc;   // GEN_ISO_ADJ_B forms wbar = rho D vbar itself
            }
        }
    }
    if (sk1) {
        float* pp = rpartial + (size_t)grp * MN + (size_t)j0 * M;
        for (int idx = threadIdx.x; idx < T * M; idx += blockDim.x) pp[idx] = acc[idx];
    }
    block_pair(racc, 0.0f, part + 2 * ((size_t)grp * gridDim.x + blockIdx.x));
}

// Iso reverse step B (grid (N / T, planes)): sbar_{k-1} = (2f - 1) wbar + (1 - f) sbar_k
// + [Nrm > tau] (tau / Nrm^3) R s_{k-1};  D^T sbar_{k-1} -> dim-1 FFT
__global__ __launch_bounds__(256) void iso_adj_b_kernel(const float* __restrict__ vbar, const float* __restrict__ sb_in,
                                                        const float* __restrict__ sk1, const float* __restrict__ nrm1,
                                                        const float* __restrict__ Rmap, float* __restrict__ sb_out,
                                                        float2* __restrict__ spec, const float2* __restrict__ twM,
                                                        FPlan pM, int N, int T, const float* __restrict__ prm) {
    const float tau = prm[0]; const float rho = prm[1];   // device-resident scalars (setup_kernel / scal_kernel)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int M = pM.n, H = M / 2 + 1;
    const size_t MN = (size_t)M * N;
    float2* A = reinterpret_cast<float2*>(smem_raw);
    float2* B = A + (size_t)((T + 1) / 2) * M;   // P = ceil(T / 2) paired transforms
    float* W0 = reinterpret_cast<float*>(B + (size_t)((T + 1) / 2) * M);
    float* W1 = W0 + (size_t)(T + 1) * M;
    const XBlk xb = xcd_block();   // XCD-aware block order (admm_kernels.hip): neighbours share L2 lines
    const int plane = xb.y, j0 = xb.x * T;
    const size_t poff = (size_t)plane * 2 * MN;
    for (int idx = threadIdx.x; idx < (T + 1) * M; idx += blockDim.x) {
        const int t = fdiv(idx, M), i = idx - t * M;
        const size_t o = (size_t)wrap(j0 + t, N) * M + i;
        const float nn = nrm1[o];
        const float f = max0_nan(1.0f - tau / nn);
        const float cw = 2.0f * f - 1.0f, cs = 1.0f - f;
        const float cf = nn > tau ? tau / (nn * nn * nn) * Rmap[o] : 0.0f;
        const float* vp = vbar + (size_t)plane * MN;
        const int j = wrap(j0 + t, N);
        const float vc = vp[o];
        const float wb[2] = {rho * (vc - vp[(size_t)wrap(j - 1, N) * M + i]), rho * (vc - vp[(size_t)j * M + wrap(i - 1, M)])};
        for (int ch = 0; ch < (t < T ? 2 : 1); ++ch) {
            const size_t q = poff + (size_t)ch * MN + o;
            const float b = sb_in ? sb_in[q] : 0.0f;
            const float r = cw * wb[ch] + cs * b + cf * sk1[q];
            (ch == 0 ? W0 : W1)[idx] = r;
            if (t < T) sb_out[q] = r;
        }
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < T * M; idx += blockDim.x) {
        const int t = fdiv(idx, M), i = idx - t * M;
        const float g = (W0[idx] - W0[idx + M]) + (W1[idx] - W1[t * M + wrap(i + 1, M)]);
        pack_real(A, t, i, M, g);
    }
    pad_odd(A, T, M);
    const float2* tw = stage_tw(smem_raw, (size_t)16 * ((T + 1) / 2) * M + (size_t)4 * (2 * T + 1) * M, twM, M);
    __syncthreads();
    const float2* R = fft<false>(A, B, (T + 1) / 2, M, pM, tw);
    store_real_spectra(R, spec + ((size_t)plane * N + j0) * H, T, M);
}

}  // namespace gen
}  // namespace admm
