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

// Aniso reverse step for T lines of one plane (grid (N / T, planes), 256 threads).
//   vb: vbar_k (spatial, HBM)    sk1: s_{k-1} (null at k = 1)   sk: s_k (null at k = K: xK used)
//   sb_in: sbar_k (null at k = K)   sb_out: sbar_{k-1}   vsum += vbar_k   spec: dim-1 FFT of D^T sbar_{k-1}
//   part: (rho_bar, tau_bar) partial of this block
__global__ __launch_bounds__(256) void line_adj_kernel(const float* __restrict__ vb, const float* __restrict__ sk1,
                                                       const float* __restrict__ sk, const float* __restrict__ xK,
                                                       const float* __restrict__ sb_in, float* __restrict__ sb_out,
                                                       float* __restrict__ vsum, float2* __restrict__ spec,
                                                       double* __restrict__ part, const float2* __restrict__ twM,
                                                       FPlan pM, int N, int Tg, const float* __restrict__ prm) {
    const float tau = prm[0]; const float rho = prm[1];   // device-resident scalars (setup_kernel)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int M = pM.n, H = M / 2 + 1;
    const size_t MN = (size_t)M * N;
    float2* A = reinterpret_cast<float2*>(smem_raw);
    float2* B = A + (size_t)((Tg + 1) / 2) * M;   // P = ceil(Tg / 2) paired transforms
    float* W0 = reinterpret_cast<float*>(B + (size_t)((Tg + 1) / 2) * M);   // sbar_{k-1} ch0, Tg+1 lines
    float* W1 = W0 + (size_t)(Tg + 1) * M;                       // sbar_{k-1} ch1, Tg lines
    float* V = reinterpret_cast<float*>(smem_raw);              // vbar lines j0-1 .. j0+T (aliases A, B)
    const XBlk xb = xcd_block();   // XCD-aware block order (admm_kernels.hip): neighbours share L2 lines
    const int plane = xb.y, j0 = xb.x * Tg;
    const int T = min(Tg, N - j0);   // the last block of a plane may be ragged (gen_nb)
    const size_t poff = (size_t)plane * 2 * MN;
    const float* vp = vb + (size_t)plane * MN;
    batched<kU>((T + 2) * M, [&](int idx) {
        const int t = fdiv(idx, M), i = idx - t * M;
        return vp[(size_t)wrap(j0 - 1 + t, N) * M + i];
    }, [&](int idx, float v) { V[idx] = v; });
    __syncthreads();
    const float* xk = (xK && !sk) ? xK + (size_t)plane * MN : nullptr;
    const float* skp = sk ? sk + poff : nullptr;
    const float* s1p = sk1 ? sk1 + poff : nullptr;
    float racc = 0.0f, tacc = 0.0f;
    struct LAdjIn {
        float a0, a1, e0, e1, e2, vs, b0, b1;
    };
    float* vsp = vsum ? vsum + (size_t)plane * MN : nullptr;   // null: neither y_bar nor h_bar wanted
    batched<kU>((T + 1) * M, [&](int idx) {
        const int t = fdiv(idx, M), i = idx - t * M;
        const int j = wrap(j0 + t, N);
        const size_t o = (size_t)j * M + i;
        const bool own = t < T;
        LAdjIn r;
        r.a0 = s1p ? s1p[o] : 0.0f;
        r.a1 = (s1p && own) ? s1p[MN + o] : 0.0f;
        r.e0 = r.e1 = r.e2 = r.vs = 0.0f;
        if (own) {   // D x_k operands (dx_at): x_K and its two neighbours, or s_k
            if (xk) {
                r.e0 = xk[o];
                r.e1 = xk[(size_t)wrap(j - 1, N) * M + i];
                r.e2 = xk[(size_t)j * M + wrap(i - 1, M)];
            } else {
                r.e0 = skp[o];
                r.e1 = skp[MN + o];
            }
            r.vs = vsp ? vsp[o] : 0.0f;
        }
        r.b0 = (s1p && sb_in) ? sb_in[poff + o] : 0.0f;
        r.b1 = (s1p && sb_in && own) ? sb_in[poff + MN + o] : 0.0f;
        return r;
    }, [&](int idx, const LAdjIn& r) {
        const int t = fdiv(idx, M), i = idx - t * M;
        const size_t o = (size_t)wrap(j0 + t, N) * M + i;
        const bool own = t < T;
        const float vc = V[(t + 1) * M + i];
        const float dv0 = vc - V[t * M + i];
        const float dv1 = vc - V[(t + 1) * M + wrap(i - 1, M)];
        if (own) {
            float d0, d1;
            if (xk) {
                d0 = r.e0 - r.e1;
                d1 = r.e0 - r.e2;
            } else {
                d0 = r.e0 - (s1p ? clip(r.a0, tau) : 0.0f);
                d1 = r.e1 - (s1p ? clip(r.a1, tau) : 0.0f);
            }
            racc -= dv0 * d0 + dv1 * d1;
            if (vsp) vsp[o] = r.vs + vc;
        }
        if (!s1p) return;   // k = 1: no sbar_0 (block-uniform)
        const float w0 = rho * dv0;
        const bool m0 = fabsf(r.a0) > tau;
        const float n0 = m0 ? w0 : r.b0 - w0;
        W0[idx] = n0;
        if (own) {
            const float w1 = rho * dv1;
            const bool m1 = fabsf(r.a1) > tau;
            const float n1 = m1 ? w1 : r.b1 - w1;
            W1[idx] = n1;
            racc += phi(r.a0, tau) * dv0 + phi(r.a1, tau) * dv1;
            tacc += (m0 ? sgn1(r.a0) * (r.b0 - 2.0f * w0) : 0.0f) + (m1 ? sgn1(r.a1) * (r.b1 - 2.0f * w1) : 0.0f);
            sb_out[poff + o] = n0;
            sb_out[poff + MN + o] = n1;
        }
    });
    block_pair(racc, tacc, part + 2 * ((size_t)plane * gridDim.x + xb.x));
    if (!s1p) return;
    __syncthreads();   // W0/W1 complete; V (aliasing A, B) is dead
    for (int idx = threadIdx.x; idx < T * M; idx += blockDim.x) {
        const int t = fdiv(idx, M), i = idx - t * M;
        const float g = (W0[idx] - W0[idx + M]) + (W1[idx] - W1[t * M + wrap(i + 1, M)]);
        pack_real(A, t, i, M, g);
    }
    pad_odd(A, T, M);
    const float2* tw = stage_tw(smem_raw, (size_t)16 * ((Tg + 1) / 2) * M + (size_t)4 * (2 * Tg + 1) * M, twM, M);
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
                                                        int M, int N, int planes, int G, int Tg, const float* __restrict__ prm) {
    const float tau = prm[0]; const float rho = prm[1];   // device-resident scalars (setup_kernel)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float* acc = reinterpret_cast<float*>(smem_raw);
    const size_t MN = (size_t)M * N;
    const int j0 = blockIdx.x * Tg, grp = blockIdx.y;
    const int T = min(Tg, N - j0);   // the last block may be ragged (gen_nb)
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
            if (vsum) vsum[(size_t)plane * MN + o] += vc;
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
                                                        FPlan pM, int N, int Tg, const float* __restrict__ prm) {
    const float tau = prm[0]; const float rho = prm[1];   // device-resident scalars (setup_kernel)
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
    const size_t poff = (size_t)plane * 2 * MN;
    struct AdjIn {
        float nn, R, vc, vu, vl, b0, b1, a0, a1;
    };
    const float* vp = vbar + (size_t)plane * MN;
    batched<kU>((T + 1) * M, [&](int idx) {
        const int t = fdiv(idx, M), i = idx - t * M;
        const int j = wrap(j0 + t, N);
        const size_t o = (size_t)j * M + i;
        AdjIn r;
        r.nn = nrm1[o];
        r.R = Rmap[o];
        r.vc = vp[o];
        r.vu = vp[(size_t)wrap(j - 1, N) * M + i];
        r.vl = vp[(size_t)j * M + wrap(i - 1, M)];
        r.b0 = sb_in ? sb_in[poff + o] : 0.0f;
        r.b1 = (sb_in && t < T) ? sb_in[poff + MN + o] : 0.0f;
        r.a0 = sk1[poff + o];
        r.a1 = t < T ? sk1[poff + MN + o] : 0.0f;
        return r;
    }, [&](int idx, const AdjIn& r) {
        const int t = fdiv(idx, M), i = idx - t * M;
        const size_t o = (size_t)wrap(j0 + t, N) * M + i;
        const float f = max0_nan(1.0f - tau / r.nn);
        const float cw = 2.0f * f - 1.0f, cs = 1.0f - f;
        const float cf = r.nn > tau ? tau / (r.nn * r.nn * r.nn) * r.R : 0.0f;
        const float r0 = cw * (rho * (r.vc - r.vu)) + cs * r.b0 + cf * r.a0;
        W0[idx] = r0;
        if (t < T) {
            const float r1 = cw * (rho * (r.vc - r.vl)) + cs * r.b1 + cf * r.a1;
            W1[idx] = r1;
            sb_out[poff + o] = r0;
            sb_out[poff + MN + o] = r1;
        }
    });
    __syncthreads();
    for (int idx = threadIdx.x; idx < T * M; idx += blockDim.x) {
        const int t = fdiv(idx, M), i = idx - t * M;
        const float g = (W0[idx] - W0[idx + M]) + (W1[idx] - W1[t * M + wrap(i + 1, M)]);
        pack_real(A, t, i, M, g);
    }
    pad_odd(A, T, M);
    const float2* tw = stage_tw(smem_raw, (size_t)16 * ((Tg + 1) / 2) * M + (size_t)4 * (2 * Tg + 1) * M, twM, M);
    __syncthreads();
    const float2* R = fft<false>(A, B, (T + 1) / 2, M, pM, tw);
    store_real_spectra(R, spec + ((size_t)plane * N + j0) * H, T, M);
}

}  // namespace gen
}  // namespace admm
