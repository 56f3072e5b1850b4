// admm_backward.hip -- adjoint of the anisotropic ADMM solve (BASELINE c5).
//
// The reference differentiates tvd_fft by letting Zygote unroll all K iterations
// (src/train.jl:51, src/ADMM_Deconv.jl:12-13), keeping every iteration's temporaries.  Here the
// forward stores one state tensor per iteration (s_k, 8 B/px) and the reverse sweep runs the same
// two-pass structure backwards (tests/kernel_model.py tvd_model_grads is the restatement, checked
// against PyTorch autograd of oracle/oracle_torch.py):
//
//   step k = K..1:  vbar_k = A^-1 g_k                       (column pass; A^-1 is symmetric)
//                   Dvb = D vbar_k
//                   rho_bar += -<Dvb, D x_k>                (x_k's dependence on rho through A)
//                   k >= 2: wbar = rho Dvb, rho_bar += <phi(s_{k-1}), Dvb>     (rho D^T w term)
//                           sbar_{k-1} = phi'(s_{k-1}) wbar + psi'(s_{k-1}) sbar_k
//                           tau_bar  += dphi/dtau wbar + dpsi/dtau sbar_k
//                           g_{k-1} = D^T sbar_{k-1}  -> rFFT along dim 1 (next column pass)
//                   Vsum += vbar_k
// with phi(s) = ST(s) - clip(s) (= z - u) and psi(s) = clip(s) (= u).  Afterwards
//   y_bar = H Vsum,   h_bar = <Vsum, dH^T y/dh> - (1/MN) sum_nu C^2 Q d|Sigma|^2/dh,
//   lam_bar = tau_bar / rho,   rho_bar -= tau_bar lam / rho^2,
// where Q[nu] = sum_k Re(conj(G_k) V_k) is accumulated by the column pass against the forward
// spectra saved in the trajectory (only when h_bar is requested).
#include <hip/hip_runtime.h>

namespace admm {

__device__ __forceinline__ float sgnf(float s) { return (s > 0.f) - (s < 0.f); }
__device__ __forceinline__ float phi_f(float s, float tau) { return fabsf(s) > tau ? s - copysignf(2.0f * tau, s) : -s; }

// block-wide reduction of two floats into doubles; lane 0 of the block writes them
__device__ __forceinline__ void block_sum2(float a, float b, double* out, double* red) {
    double da = a, db = b;
    for (int off = 32; off > 0; off >>= 1) {
        da += __shfl_down(da, off);
        db += __shfl_down(db, off);
    }
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) { red[2 * w] = da; red[2 * w + 1] = db; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double sa = 0.0, sb = 0.0;
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) { sa += red[2 * i]; sb += red[2 * i + 1]; }
        out[0] = sa;
        out[1] = sb;
    }
}

// ----------------------------------------------------------------------------------------------
// LINE_ADJ: one reverse step's line work for T lines (+1 halo line each side of vbar).
//   spec1  : line spectrum of vbar_k (output of the adjoint column pass)
//   sk1    : s_{k-1} (trajectory; null for k = 1)      sk : s_k (null for k = K)
//   xK     : forward output x_K (used only at k = K for D x_K)
//   sb_in  : sbar_k (null at k = K: zero)              sb_out : sbar_{k-1}
//   vsum   : running sum of vbar (read-modify-write)   spec0 : rFFT_dim1 of g_{k-1}
//   part   : per-block (rho_bar, tau_bar) partial sums
// ----------------------------------------------------------------------------------------------
// s of 4 pixels (i..i+3 of line j), both channels, from a plane's trajectory slot: the 2-pass layout
// [ch][N][M], or (LN) the fused kernel's lane-native layout (plane_api.hpp: float4 (s0[p], s0[p+1],
// s1[p], s1[p+1]) of pixel pair p = 4n + 2h of line j at [n][2j + h], M = 256)
template <bool LN>
__device__ __forceinline__ void load_s_quad(const float* __restrict__ sp, int j, int i, int M, size_t MN, bool c1_too,
                                            float (&c0)[4], float (&c1)[4]) {
    if constexpr (LN) {
        const float4* q = reinterpret_cast<const float4*>(sp) + (size_t)(i >> 2) * 512 + 2 * j;
        const float4 a = q[0], b = q[1];
        c0[0] = a.x; c0[1] = a.y; c0[2] = b.x; c0[3] = b.y;
        c1[0] = a.z; c1[1] = a.w; c1[2] = b.z; c1[3] = b.w;
    } else {
        const float4 a = *reinterpret_cast<const float4*>(sp + (size_t)j * M + i);
        c0[0] = a.x; c0[1] = a.y; c0[2] = a.z; c0[3] = a.w;
        if (c1_too) {
            const float4 b = *reinterpret_cast<const float4*>(sp + MN + (size_t)j * M + i);
            c1[0] = b.x; c1[1] = b.y; c1[2] = b.z; c1[3] = b.w;
        }
    }
}

template <int L, int T, bool LN = false>
__global__ __launch_bounds__(kThreads) void line_adj_kernel(const float2* __restrict__ spec1,
                                                            const float* __restrict__ sk1, const float* __restrict__ sk,
                                                            const float* __restrict__ xK,
                                                            const float* __restrict__ sb_in, float* __restrict__ sb_out,
                                                            float* __restrict__ vsum, float2* __restrict__ spec0,
                                                            double* __restrict__ part, const float2* __restrict__ twM,
                                                            int N, const float* __restrict__ prm, int first_k /*k==1*/,
                                                            int last_k /*k==K*/, Branches br = kOneSolve, size_t pbs = 0) {
    // several branches (admm_kernels.hip Branches): own scalars, x_K in the chcat layout, the partial rows of
    // branch i pbs doubles on, rows by the plane's index within its branch
    constexpr int M = 2 * L;
    constexpr int M4 = M / 4;
    constexpr int TH = T + 2;
    constexpr int P = Plan<L>::P;
    constexpr int RF = plan_radix<L, 0, true>();
    constexpr int QF = L / RF;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float2* tw = reinterpret_cast<float2*>(smem_raw);
    float2* X = tw + M;
    float2* Bf = X + TH * L;
    float2* Cf = Bf + TH * L;
    double* red = reinterpret_cast<double*>(Cf + TH * L);   // 2 doubles per wave
    const XBlk xb = xcd_block();
    const int plane = xb.y;
    const int j0 = xb.x * T;
    const size_t MN = (size_t)M * N;
    const int tid = threadIdx.x;
    const size_t poff = (size_t)plane * 2 * MN;
    const BranchOf bo = branch_of(br, plane);
    const float tau = prm[(size_t)bo.i * br.prm_f], rho = prm[(size_t)bo.i * br.prm_f + 1];   // (setup_kernel)

    for (int t = tid; t < M; t += kThreads) tw[t] = twM[t];
    load_lines<L>(spec1 + (size_t)plane * N * L, X, j0 - 1, TH, N);
    __syncthreads();
    auto uload = [&](int f, int n) { return unpack_z<L>(X + f * L, n, tw); };
    float2* Xr;
    if constexpr (P == 1) {
        Xr = Bf;
        fpass<L, L, 0, true, 2>(TH, tw, uload, LdsIO{Bf, L});
    } else if constexpr (P == 2) {
        Xr = X;
        fft_plan<L, false, true, 2>(TH, tw, Bf, Cf, L, uload, LdsIO{X, L});
    } else {
        Xr = Bf;
        plan_pass<L, 0, false, true, 2>(TH, tw, uload, LdsIO{Bf, L});
        __syncthreads();
        plan_pass<L, 1, false, true, 2>(TH, tw, LdsIO{Bf, L}, LdsIO{Cf, L});
        __syncthreads();
        plan_pass<L, 2, false, true, 2>(TH, tw, LdsIO{Cf, L}, LdsIO{Bf, L});
    }
    __syncthreads();
    const float* vb = reinterpret_cast<const float*>(Xr);       // vbar lines j0-1 .. j0+T
    float* SB0 = reinterpret_cast<float*>(Xr == X ? Bf : X);    // sbar_{k-1} ch0, lines j0..j0+T
    float* SB1 = reinterpret_cast<float*>(Cf);                  // sbar_{k-1} ch1, lines j0..j0+T-1

    float rho_acc = 0.0f, tau_acc = 0.0f;
    for (int idx = tid; idx < (T + 1) * M4; idx += kThreads) {
        const int t = idx / M4;
        const int i = (idx - t * M4) * 4;
        const size_t off = (size_t)((j0 + t) & (N - 1)) * M + i;
        const float4 vc = *reinterpret_cast<const float4*>(vb + (t + 1) * M + i);
        const float4 vp = *reinterpret_cast<const float4*>(vb + t * M + i);
        const float vl = vb[(t + 1) * M + ((i - 1) & (M - 1))];
        const float dv0[4] = {vc.x - vp.x, vc.y - vp.y, vc.z - vp.z, vc.w - vp.w};
        const float dv1[4] = {vc.x - vl, vc.y - vc.x, vc.z - vc.y, vc.w - vc.z};
        const bool own = t < T;
        float s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0};   // s_{k-1}
        if (!first_k) {
            load_s_quad<LN>(sk1 + poff, (j0 + t) & (N - 1), i, M, MN, own, s0, s1);
            if (!own) s1[0] = s1[1] = s1[2] = s1[3] = 0.0f;
        }
        if (own) {
            // ---- rho_bar: -<Dvb, D x_k> (xK / sk null: rho_bar not wanted, no reads) ----
            float dx0[4] = {0, 0, 0, 0}, dx1[4] = {0, 0, 0, 0};
            if (last_k && xK) {
                const float* xp = xK + bo.out_plane * MN;
                const float4 xc = *reinterpret_cast<const float4*>(xp + off);
                const float4 xq = *reinterpret_cast<const float4*>(xp + (size_t)((j0 + t - 1) & (N - 1)) * M + i);
                const float xl = xp[(size_t)((j0 + t) & (N - 1)) * M + ((i - 1) & (M - 1))];
                dx0[0] = xc.x - xq.x; dx0[1] = xc.y - xq.y; dx0[2] = xc.z - xq.z; dx0[3] = xc.w - xq.w;
                dx1[0] = xc.x - xl; dx1[1] = xc.y - xc.x; dx1[2] = xc.z - xc.y; dx1[3] = xc.w - xc.z;
            } else if (!last_k && sk) {
                float a4[4], b4[4];
                load_s_quad<LN>(sk + poff, (j0 + t) & (N - 1), i, M, MN, true, a4, b4);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    dx0[q] = a4[q] - fminf(fmaxf(s0[q], -tau), tau);
                    dx1[q] = b4[q] - fminf(fmaxf(s1[q], -tau), tau);
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) rho_acc -= dv0[q] * dx0[q] + dv1[q] * dx1[q];
            // ---- Vsum += vbar (null: neither y_bar nor h_bar wanted) ----
            if (vsum) {
                float4* vs = reinterpret_cast<float4*>(vsum + (size_t)plane * MN + off);
                float4 acc = *vs;
                acc.x += vc.x; acc.y += vc.y; acc.z += vc.z; acc.w += vc.w;
                *vs = acc;
            }
        }
        if (!first_k) {
            float sb0[4] = {0, 0, 0, 0}, sb1[4] = {0, 0, 0, 0};   // sbar_k
            if (sb_in) {
                const float4 a = *reinterpret_cast<const float4*>(sb_in + poff + off);
                sb0[0] = a.x; sb0[1] = a.y; sb0[2] = a.z; sb0[3] = a.w;
                if (own) {
                    const float4 b = *reinterpret_cast<const float4*>(sb_in + poff + MN + off);
                    sb1[0] = b.x; sb1[1] = b.y; sb1[2] = b.z; sb1[3] = b.w;
                }
            }
            float n0[4], n1[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float wb = rho * dv0[q];
                const bool m = fabsf(s0[q]) > tau;
                n0[q] = m ? wb : sb0[q] - wb;
                if (own) {
                    rho_acc += phi_f(s0[q], tau) * dv0[q];
                    if (m) tau_acc += sgnf(s0[q]) * (sb0[q] - 2.0f * wb);
                }
            }
            *reinterpret_cast<float4*>(SB0 + t * M + i) = make_float4(n0[0], n0[1], n0[2], n0[3]);
            if (own) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float wb = rho * dv1[q];
                    const bool m = fabsf(s1[q]) > tau;
                    n1[q] = m ? wb : sb1[q] - wb;
                    rho_acc += phi_f(s1[q], tau) * dv1[q];
                    if (m) tau_acc += sgnf(s1[q]) * (sb1[q] - 2.0f * wb);
                }
                *reinterpret_cast<float4*>(SB1 + t * M + i) = make_float4(n1[0], n1[1], n1[2], n1[3]);
                *reinterpret_cast<float4*>(sb_out + poff + off) = make_float4(n0[0], n0[1], n0[2], n0[3]);
                *reinterpret_cast<float4*>(sb_out + poff + MN + off) = make_float4(n1[0], n1[1], n1[2], n1[3]);
            }
        }
    }
    block_sum2(rho_acc, tau_acc, part + (size_t)bo.i * pbs + 2 * (bo.in_plane * gridDim.x + xb.x), red);
    if (first_k) return;   // k = 1: no g_0 (block-uniform)
    __syncthreads();
    // ---- g_{k-1} = D^T sbar_{k-1}, fed straight into the forward pass 0 along dim 1 ----
    float2* F0 = const_cast<float2*>(reinterpret_cast<const float2*>(vb));   // vbar dead now
    for (int idx = tid; idx < T * QF; idx += kThreads) {
        const int f = idx / QF, j = idx - f * QF;
        float2 v[RF];
#pragma unroll
        for (int r = 0; r < RF; ++r) {
            const int n = j + r * QF;
            const float2 a = *reinterpret_cast<const float2*>(SB0 + f * M + 2 * n);
            const float2 b = *reinterpret_cast<const float2*>(SB0 + (f + 1) * M + 2 * n);
            const float2 c = *reinterpret_cast<const float2*>(SB1 + f * M + 2 * n);
            const float cn = SB1[f * M + ((2 * n + 2) & (M - 1))];
            v[r].x = (a.x - b.x) + (c.x - c.y);
            v[r].y = (a.y - b.y) + (c.y - cn);
        }
        fly_core<L, RF, 0, false, 2>(v, j, tw);
        const int o = out_base<L, RF, 0>(j);
#pragma unroll
        for (int r = 0; r < RF; ++r) F0[f * L + o + r] = v[r];
    }
    __syncthreads();
    float2* Z;
    if constexpr (P == 1) {
        Z = F0;
    } else if constexpr (P == 2) {
        float2* Zb = reinterpret_cast<float2*>(SB0);
        plan_pass<L, 1, true, false, 2>(T, tw, LdsIO{F0, L}, LdsIO{Zb, L});
        __syncthreads();
        Z = Zb;
    } else {
        float2* Zb = reinterpret_cast<float2*>(SB0);
        plan_pass<L, 1, true, false, 2>(T, tw, LdsIO{F0, L}, LdsIO{Zb, L});
        __syncthreads();
        plan_pass<L, 2, true, false, 2>(T, tw, LdsIO{Zb, L}, LdsIO{F0, L});
        __syncthreads();
        Z = F0;
    }
    pack_store<L>(Z, spec0 + (size_t)plane * N * L, j0, T, N, tw);
}

// h_bar through H^T y: hb[b][a] = sum_planes sum_px Vsum[j][i] * y[j+b-padr][i+a-padd]  (one block per
// (plane, line tile); per-tap partials, deterministic order).  Tile of TY lines, y halo in LDS.
__global__ __launch_bounds__(kThreads) void hbar_corr_kernel(const float* __restrict__ vsum, const float* __restrict__ y,
                                                             double* __restrict__ part, int M, int N, int kh, int kw,
                                                             int TY) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float* Vt = reinterpret_cast<float*>(smem_raw);        // TY lines
    float* Yt = Vt + (size_t)TY * M;                        // TY + kw - 1 lines
    const int plane = blockIdx.y;
    const int j0 = blockIdx.x * TY;
    const int padd = (kh - 1) / 2, padr = (kw - 1) / 2;
    const size_t MN = (size_t)M * N;
    const float* vp = vsum + (size_t)plane * MN;
    const float* yp = y + (size_t)plane * MN;
    for (int idx = threadIdx.x; idx < TY * M; idx += blockDim.x) Vt[idx] = vp[(size_t)j0 * M + idx];
    for (int idx = threadIdx.x; idx < (TY + kw - 1) * M; idx += blockDim.x) {
        const int r = idx / M, i = idx - r * M;
        int jj = (j0 - padr + r) % N;   // any N (the runtime-length path too); kw <= N
        jj += jj < 0 ? N : 0;
        Yt[idx] = yp[(size_t)jj * M + i];
    }
    __syncthreads();
    const int ntaps = kh * kw;
    double* out = part + ((size_t)plane * gridDim.x + blockIdx.x) * ntaps;
    // one wave per tap at a time: lanes stride over the tile's pixels
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    for (int tap = wave; tap < ntaps; tap += nw) {
        const int b = tap / kh, a = tap - b * kh;
        double d = 0.0;   // fp64 per lane: TY * M / 64 products each
        for (int p = lane; p < TY * M; p += 64) {
            const int t = p / M, i = p - t * M;
            int ii = i + a - padd;   // in (-M, 2M) for kh <= M
            ii += ii < 0 ? M : 0;
            ii -= ii >= M ? M : 0;
            d += (double)Vt[p] * Yt[(t + b) * M + ii];
        }
        for (int off = 32; off > 0; off >>= 1) d += __shfl_down(d, off);
        if (lane == 0) out[tap] = d;
    }
}

// Sum column c (= blockIdx.x) of an n x w row-major matrix of per-block partials, in a fixed order.
// first stage of a long column sum: block (c, g) sums rows [g chunk, (g + 1) chunk) of column c into
// tmp[g w + c] (fixed partition: deterministic); reduce_cols_kernel then sums the gridDim.y partials
__global__ __launch_bounds__(kThreads) void reduce_cols_part_kernel(const double* __restrict__ part,
                                                                    double* __restrict__ tmp, int n, int w, int chunk) {
    __shared__ double red[kThreads];
    const int c = blockIdx.x, g = blockIdx.y;
    const int i0 = g * chunk, i1 = min(n, i0 + chunk);
    double s = 0.0;
    for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) s += part[(size_t)i * w + c];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int off = blockDim.x / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x == 0) tmp[(size_t)g * w + c] = red[0];
}

__global__ __launch_bounds__(kThreads) void reduce_cols_kernel(const double* __restrict__ part,
                                                               double* __restrict__ out, int n, int w) {
    __shared__ double red[kThreads];
    const int c = blockIdx.x;
    double s = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) s += part[(size_t)i * w + c];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int off = blockDim.x / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[c] = red[0];
}

// h_bar through A (needs Q): hbA[b][a] = -(1/MN) sum_{kj, k=0..L} w_k C^2 Q d|Sigma|^2/dh[b][a],
// d|Sigma|^2/dh = 2 Re(conj(Sigma) e^{-2 pi i (a k/M + b kj/N)}); Sigma rebuilt in fp64.  One block per tap.
__global__ __launch_bounds__(kThreads) void hbarA_kernel(const double* __restrict__ Q, const float* __restrict__ Ct,
                                                         const double2* __restrict__ SigT, int kh, int M, int N,
                                                         double* __restrict__ out) {
    __shared__ double red[kThreads / 64];
    const int tap = blockIdx.x;
    const int b = tap / kh, a = tap - b * kh;
    const int L = M / 2, H = L + 1;
    double acc = 0.0;
    for (int q = threadIdx.x; q < H * N; q += blockDim.x) {
        const int kj = q / H, k = q - kj * H;
        double s, c;
        sincospi(-2.0 * ((double)((a * k) % M) / M + (double)((b * kj) % N) / N), &s, &c);
        const double2 S = SigT[q];
        const double dS = 2.0 * (S.x * c + S.y * s);    // 2 Re(conj(Sigma) e^{-i th})
        const double Cm = (double)Ct[q] * (double)M * (double)N;   // Ct holds C/(MN)
        const double wk = (k == 0 || 2 * k == M) ? 1.0 : 2.0;   // self-conjugate bins (M odd: bin 0 only)
        acc += wk * Cm * Cm * Q[q] * dS;
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) red[w] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double sum = 0.0;
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) sum += red[i];
        out[tap] = -sum / ((double)M * (double)N);
    }
}

// Q[q] = sum over planes of Qp[p][q] (fixed order, fp64)
__global__ void reduce_planes_kernel(const double* __restrict__ Qp, double* __restrict__ Q, int planes, int n) {
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) {
        double s = 0.0;
        for (int p = 0; p < planes; ++p) s += Qp[(size_t)p * n + q];
        Q[q] = s;
    }
}

// Final assembly of the scalar / PSF gradients into the caller's fp32 outputs.
__global__ void grads_final_kernel(const double* __restrict__ rt, const double* __restrict__ hb_corr,
                                   const double* __restrict__ hb_A, int ntaps, const float* __restrict__ prm,
                                   float* __restrict__ lam_bar, float* __restrict__ rho_bar, float* __restrict__ h_bar) {
    const float lam = prm[2]; const float rho = prm[1];   // device-resident scalars (setup_kernel)
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t == 0) {
        const double tau_bar = rt[1];
        if (lam_bar) *lam_bar = (float)(tau_bar / rho);
        if (rho_bar) *rho_bar = (float)(rt[0] - tau_bar * lam / ((double)rho * rho));
    }
    if (h_bar && t < ntaps) h_bar[t] = (float)(hb_corr[t] + (hb_A ? hb_A[t] : 0.0));
}


// ==============================================================================================
// Isotropic (BT) adjoint (tests/kernel_model.py tvd_model_grads(iso=True) is the restatement).
// With f = max(1 - tau/Nrm, 0), Nrm(pixel) = sqrt(sum over ALL planes and both channels of s^2):
// w = (2f - 1) s, u = (1 - f) s, and one reverse step needs the batch reduction
//   R(pixel) = sum_{planes, channels} s_{k-1} (2 wbar - sbar_k),   wbar = rho D vbar_k
//   sbar_{k-1} = (2f - 1) wbar + (1 - f) sbar_k + [Nrm > tau] (tau / Nrm^3) R s_{k-1}
//   tau_bar  += sum_pixels [Nrm > tau] (-R / Nrm)
// so the step runs as ISO_ADJ_A (per plane group: vbar, D vbar, rho_bar, Vsum, wbar, partial R) ->
// ISO_ADJ_R (R map, tau_bar) -> ISO_ADJ_B (per plane: sbar_{k-1}, D^T, rFFT) -- the forward's
// iso_a -> iso_r -> iso_b shape.  nrm1 is the saved Nrm of iteration k-1.
// ==============================================================================================
__device__ __forceinline__ float bt_factor(float nrm, float tau) { return max0_nan(1.0f - tau / nrm); }

template <int L, int T>
__global__ __launch_bounds__(kThreads) void iso_adj_a_kernel(const float2* __restrict__ spec1,
                                                             const float* __restrict__ sk1, const float* __restrict__ sk,
                                                             const float* __restrict__ xK,
                                                             const float* __restrict__ nrm1, const float* __restrict__ nrm0,
                                                             const float* __restrict__ sb_in, float* __restrict__ vbar_out,
                                                             float* __restrict__ vsum, float* __restrict__ rpartial,
                                                             double* __restrict__ part, const float2* __restrict__ twM,
                                                             int N, int planes, int G, const float* __restrict__ prm,
                                                             int first_k, int last_k, Branches br = kOneSolve,
                                                             int ngb = 0, size_t pbs = 0) {
    // several branches (admm_kernels.hip Branches): planes per branch, ngb plane groups per branch (grid y =
    // branches x ngb), pbs doubles between the branches' partial-row blocks; xK in the chcat layout
    // nrm1 = Nrm_{k-1} (k >= 2), nrm0 = Nrm_{k-2} (k >= 3; for D x_k = s_k - psi(s_{k-1}) we need f_{k-1}
    // only: nrm0 is unused but kept for symmetry of the call -- psi(s_{k-1}) uses nrm1)
    (void)nrm0;
    constexpr int M = 2 * L;
    constexpr int M4 = M / 4;
    constexpr int TH = T + 1;
    constexpr int NE = T * M4;
    constexpr int NIT = (NE + kThreads - 1) / kThreads;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float2* tw = reinterpret_cast<float2*>(smem_raw);
    float2* X = tw + M;
    float2* Bf = X + TH * L;
    float2* Cf = Bf + TH * L;
    double* red = reinterpret_cast<double*>(Cf + TH * L);
    const XBlk xb = xcd_block();
    const int j0 = xb.x * T;
    const int grp = xb.y;
    const int nb_ = ngb > 0 ? ngb : (int)gridDim.y;
    const int bri = grp / nb_, gl = grp - bri * nb_;
    const size_t MN = (size_t)M * N;
    if (nrm1) nrm1 += (size_t)bri * MN;
    prm += (size_t)bri * br.prm_f;
    part += (size_t)bri * pbs;
    const float tau = prm[0]; const float rho = prm[1];   // device-resident scalars (setup_kernel)
    const int tid = threadIdx.x;
    for (int t = tid; t < M; t += kThreads) tw[t] = twM[t];
    float4 racc[NIT], fo[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
        racc[it] = make_float4(0.f, 0.f, 0.f, 0.f);
        fo[it] = make_float4(0.f, 0.f, 0.f, 0.f);
        const int idx = tid + it * kThreads;
        if (!first_k && idx < NE) {
            const int t = idx / M4, i = (idx - t * M4) * 4;
            const float4 nn = *reinterpret_cast<const float4*>(nrm1 + (size_t)(j0 + t) * M + i);
            fo[it] = make_float4(bt_factor(nn.x, tau), bt_factor(nn.y, tau), bt_factor(nn.z, tau), bt_factor(nn.w, tau));
        }
    }
    float rho_acc = 0.0f;
    const int p_end = bri * planes + min(planes, (gl + 1) * G);
    for (int plane = bri * planes + gl * G; plane < p_end; ++plane) {
        __syncthreads();
        load_lines<L>(spec1 + (size_t)plane * N * L, X, j0 - 1, TH, N);
        __syncthreads();
        auto uload = [&](int f, int n) { return unpack_z<L>(X + f * L, n, tw); };
        float2* Xr;
        if constexpr (Plan<L>::P == 1) {
            Xr = Bf;
            fpass<L, L, 0, true, 2>(TH, tw, uload, LdsIO{Bf, L});
        } else if constexpr (Plan<L>::P == 2) {
            Xr = X;
            fft_plan<L, false, true, 2>(TH, tw, Bf, Cf, L, uload, LdsIO{X, L});
        } else {
            Xr = Bf;
            plan_pass<L, 0, false, true, 2>(TH, tw, uload, LdsIO{Bf, L});
            __syncthreads();
            plan_pass<L, 1, false, true, 2>(TH, tw, LdsIO{Bf, L}, LdsIO{Cf, L});
            __syncthreads();
            plan_pass<L, 2, false, true, 2>(TH, tw, LdsIO{Cf, L}, LdsIO{Bf, L});
        }
        __syncthreads();
        const float* vb = reinterpret_cast<const float*>(Xr);   // lines j0-1 .. j0+T-1
        const size_t poff = (size_t)plane * 2 * MN;
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int idx = tid + it * kThreads;
            if (idx >= NE) continue;
            const int t = idx / M4, i = (idx - t * M4) * 4;
            const size_t off = (size_t)(j0 + t) * M + i;
            const float4 vc = *reinterpret_cast<const float4*>(vb + (t + 1) * M + i);
            const float4 vp = *reinterpret_cast<const float4*>(vb + t * M + i);
            const float vl = vb[(t + 1) * M + ((i - 1) & (M - 1))];
            const float dv0[4] = {vc.x - vp.x, vc.y - vp.y, vc.z - vp.z, vc.w - vp.w};
            const float dv1[4] = {vc.x - vl, vc.y - vc.x, vc.z - vc.y, vc.w - vc.z};
            const float f4[4] = {fo[it].x, fo[it].y, fo[it].z, fo[it].w};
            float a0[4] = {0, 0, 0, 0}, a1[4] = {0, 0, 0, 0};   // s_{k-1}
            if (!first_k) {
                const float4 a = *reinterpret_cast<const float4*>(sk1 + poff + off);
                const float4 b = *reinterpret_cast<const float4*>(sk1 + poff + MN + off);
                a0[0] = a.x; a0[1] = a.y; a0[2] = a.z; a0[3] = a.w;
                a1[0] = b.x; a1[1] = b.y; a1[2] = b.z; a1[3] = b.w;
            }
            // ---- rho_bar: -<D vbar, D x_k> ----
            // (xK / sk null: rho_bar not wanted, D x_k reads as 0 and costs no traffic)
            float dx0[4] = {0, 0, 0, 0}, dx1[4] = {0, 0, 0, 0};
            if (last_k && xK) {
                const float* xp = xK + branch_of(br, plane).out_plane * MN;
                const float4 xc = *reinterpret_cast<const float4*>(xp + off);
                const float4 xq = *reinterpret_cast<const float4*>(xp + (size_t)((j0 + t - 1) & (N - 1)) * M + i);
                const float xl = xp[(size_t)(j0 + t) * M + ((i - 1) & (M - 1))];
                dx0[0] = xc.x - xq.x; dx0[1] = xc.y - xq.y; dx0[2] = xc.z - xq.z; dx0[3] = xc.w - xq.w;
                dx1[0] = xc.x - xl; dx1[1] = xc.y - xc.x; dx1[2] = xc.z - xc.y; dx1[3] = xc.w - xc.z;
            } else if (!last_k && sk) {
                const float4 a = *reinterpret_cast<const float4*>(sk + poff + off);
                const float4 b = *reinterpret_cast<const float4*>(sk + poff + MN + off);
                const float c0[4] = {a.x, a.y, a.z, a.w}, c1[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {   // D x_k = s_k - psi(s_{k-1}) = s_k - (1 - f_{k-1}) s_{k-1}
                    dx0[q] = c0[q] - (1.0f - f4[q]) * a0[q];
                    dx1[q] = c1[q] - (1.0f - f4[q]) * a1[q];
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) rho_acc -= dv0[q] * dx0[q] + dv1[q] * dx1[q];
            if (vsum) {   // null: neither y_bar nor h_bar wanted
                float4* vs = reinterpret_cast<float4*>(vsum + (size_t)plane * MN + off);
                float4 acc = *vs;
                acc.x += vc.x; acc.y += vc.y; acc.z += vc.z; acc.w += vc.w;
                *vs = acc;
            }
            if (!first_k) {
                // vbar_k for ISO_ADJ_B, which forms wbar = rho D vbar itself (4 B/px here and ~5 there,
                // against 8 + 8 for a stored two-channel wbar)
                *reinterpret_cast<float4*>(vbar_out + (size_t)plane * MN + off) = vc;
                float b0[4] = {0, 0, 0, 0}, b1[4] = {0, 0, 0, 0};   // sbar_k
                if (sb_in) {
                    const float4 a = *reinterpret_cast<const float4*>(sb_in + poff + off);
                    const float4 b = *reinterpret_cast<const float4*>(sb_in + poff + MN + off);
                    b0[0] = a.x; b0[1] = a.y; b0[2] = a.z; b0[3] = a.w;
                    b1[0] = b.x; b1[1] = b.y; b1[2] = b.z; b1[3] = b.w;
                }
                float w0[4], w1[4], rr[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    w0[q] = rho * dv0[q];
                    w1[q] = rho * dv1[q];
                    const float ph = 2.0f * f4[q] - 1.0f;   // phi(s) = (2f - 1) s
                    rho_acc += ph * (a0[q] * dv0[q] + a1[q] * dv1[q]);
                    rr[q] = a0[q] * (2.0f * w0[q] - b0[q]) + a1[q] * (2.0f * w1[q] - b1[q]);
                }

                racc[it].x += rr[0]; racc[it].y += rr[1]; racc[it].z += rr[2]; racc[it].w += rr[3];
            }
        }
    }
    if (!first_k) {
        float* pp = rpartial + (size_t)grp * MN;
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int idx = tid + it * kThreads;
            if (idx < NE) {
                const int t = idx / M4, i = (idx - t * M4) * 4;
                *reinterpret_cast<float4*>(pp + (size_t)(j0 + t) * M + i) = racc[it];
            }
        }
    }
    __syncthreads();
    block_sum2(rho_acc, 0.0f, part + 2 * ((size_t)gl * gridDim.x + xb.x), red);
}

// R map = sum over plane groups of the partial sums; tau_bar partials (block-reduced, one pair per block)
// grid (blocks, branches): branch blockIdx.y sums its own ngroups partials; its tau_bar rows pbs doubles on
__global__ __launch_bounds__(kThreads) void iso_adj_r_kernel(const float* __restrict__ rpartial, float* __restrict__ Rmap,
                                                             const float* __restrict__ nrm1, int ngroups, size_t MN,
                                                             const float* __restrict__ prm, double* __restrict__ part,
                                                             unsigned prm_f = 0, size_t pbs = 0) {
    const size_t bi = blockIdx.y;
    rpartial += bi * ngroups * MN;
    Rmap += bi * MN;
    nrm1 += bi * MN;
    part += bi * pbs;
    const float tau = prm[bi * prm_f];   // device-resident scalars (setup_kernel)
    __shared__ double red[2 * (kThreads / 64)];
    __shared__ float gred[kThreads];
    float tacc = 0.0f;
    for (size_t base = (size_t)blockIdx.x * 64; base < MN; base += (size_t)gridDim.x * 64) {
        const size_t q = base + (threadIdx.x & 63);
        const float R = group_sum(rpartial, ngroups, MN, q, gred);   // group_sum: admm_kernels.hip
        if (threadIdx.x < 64 && q < MN) {
            Rmap[q] = R;
            const float nn = nrm1[q];
            if (nn > tau) tacc -= R / nn;
        }
    }
    block_sum2(0.0f, tacc, part + 2 * blockIdx.x, red);
}

// sbar_{k-1} = (2f - 1) wbar + (1 - f) sbar_k + [Nrm > tau] (tau/Nrm^3) R s_{k-1}; g = D^T sbar -> rFFT
template <int L, int T>
__global__ __launch_bounds__(kThreads) void iso_adj_b_kernel(const float* __restrict__ vbar, const float* __restrict__ sb_in,
                                                             const float* __restrict__ sk1, const float* __restrict__ nrm1,
                                                             const float* __restrict__ Rmap, float* __restrict__ sb_out,
                                                             float2* __restrict__ spec0, const float2* __restrict__ twM,
                                                             int N, const float* __restrict__ prm, Branches br = kOneSolve) {
    constexpr int M = 2 * L;
    constexpr int M4 = M / 4;
    constexpr int P = Plan<L>::P;
    constexpr int RF = plan_radix<L, 0, true>();
    constexpr int QF = L / RF;
    constexpr int NE = (T + 1) * M4;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float2* tw = reinterpret_cast<float2*>(smem_raw);
    float* W0 = reinterpret_cast<float*>(tw + M);   // sbar ch0, T+1 lines
    float* W1 = W0 + (T + 1) * M;                   // sbar ch1, T lines
    float2* F0 = reinterpret_cast<float2*>(W1 + T * M);
    float2* F1 = F0 + T * L;
    const XBlk xb = xcd_block();
    const int plane = xb.y;
    const int j0 = xb.x * T;
    const size_t MN = (size_t)M * N;
    const int tid = threadIdx.x;
    const size_t poff = (size_t)plane * 2 * MN;
    const int bri = branch_of(br, plane).i;
    nrm1 += (size_t)bri * MN;
    Rmap += (size_t)bri * MN;
    const float tau = prm[(size_t)bri * br.prm_f], rho = prm[(size_t)bri * br.prm_f + 1];   // (setup_kernel)
    for (int t = tid; t < M; t += kThreads) tw[t] = twM[t];
    for (int idx = tid; idx < NE; idx += kThreads) {
        const int t = idx / M4, i = (idx - t * M4) * 4;
        const size_t off = (size_t)((j0 + t) & (N - 1)) * M + i;
        const float4 nn = *reinterpret_cast<const float4*>(nrm1 + off);
        const float4 R = *reinterpret_cast<const float4*>(Rmap + off);
        const float n4[4] = {nn.x, nn.y, nn.z, nn.w}, r4[4] = {R.x, R.y, R.z, R.w};
        float cf[4], cw[4], cs[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float f = bt_factor(n4[q], tau);
            cw[q] = 2.0f * f - 1.0f;
            cs[q] = 1.0f - f;
            cf[q] = n4[q] > tau ? tau / (n4[q] * n4[q] * n4[q]) * r4[q] : 0.0f;
        }
        // wbar = rho D vbar_k, bitwise as ISO_ADJ_A formed it
        const float* vp = vbar + (size_t)plane * MN;
        const float4 vc = *reinterpret_cast<const float4*>(vp + off);
        const float4 vu = *reinterpret_cast<const float4*>(vp + (size_t)((j0 + t - 1) & (N - 1)) * M + i);
        const float vl = vp[(size_t)((j0 + t) & (N - 1)) * M + ((i - 1) & (M - 1))];
        const float4 wb0 = make_float4(rho * (vc.x - vu.x), rho * (vc.y - vu.y), rho * (vc.z - vu.z), rho * (vc.w - vu.w));
        const float4 wb1 = make_float4(rho * (vc.x - vl), rho * (vc.y - vc.x), rho * (vc.z - vc.y), rho * (vc.w - vc.z));
        for (int ch = 0; ch < (t < T ? 2 : 1); ++ch) {
            const size_t o = poff + (size_t)ch * MN + off;
            const float4 w = ch == 0 ? wb0 : wb1;
            const float4 a = *reinterpret_cast<const float4*>(sk1 + o);
            float4 b = make_float4(0.f, 0.f, 0.f, 0.f);
            if (sb_in) b = *reinterpret_cast<const float4*>(sb_in + o);
            float4 r;
            r.x = cw[0] * w.x + cs[0] * b.x + cf[0] * a.x;
            r.y = cw[1] * w.y + cs[1] * b.y + cf[1] * a.y;
            r.z = cw[2] * w.z + cs[2] * b.z + cf[2] * a.z;
            r.w = cw[3] * w.w + cs[3] * b.w + cf[3] * a.w;
            *reinterpret_cast<float4*>((ch == 0 ? W0 : W1) + t * M + i) = r;
            if (t < T) *reinterpret_cast<float4*>(sb_out + o) = r;
        }
    }
    __syncthreads();
    for (int idx = tid; idx < T * QF; idx += kThreads) {
        const int f = idx / QF, j = idx - f * QF;
        float2 v[RF];
#pragma unroll
        for (int r = 0; r < RF; ++r) {
            const int n = j + r * QF;
            const float2 a = *reinterpret_cast<const float2*>(W0 + f * M + 2 * n);
            const float2 b = *reinterpret_cast<const float2*>(W0 + (f + 1) * M + 2 * n);
            const float2 c = *reinterpret_cast<const float2*>(W1 + f * M + 2 * n);
            const float cn = W1[f * M + ((2 * n + 2) & (M - 1))];
            v[r].x = (a.x - b.x) + (c.x - c.y);
            v[r].y = (a.y - b.y) + (c.y - cn);
        }
        fly_core<L, RF, 0, false, 2>(v, j, tw);
        const int o = out_base<L, RF, 0>(j);
#pragma unroll
        for (int r = 0; r < RF; ++r) F0[f * L + o + r] = v[r];
    }
    __syncthreads();
    float2* Z;
    if constexpr (P == 1) {
        Z = F0;
    } else if constexpr (P == 2) {
        plan_pass<L, 1, true, false, 2>(T, tw, LdsIO{F0, L}, LdsIO{F1, L});
        __syncthreads();
        Z = F1;
    } else {
        plan_pass<L, 1, true, false, 2>(T, tw, LdsIO{F0, L}, LdsIO{F1, L});
        __syncthreads();
        plan_pass<L, 2, true, false, 2>(T, tw, LdsIO{F1, L}, LdsIO{F0, L});
        __syncthreads();
        Z = F0;
    }
    pack_store<L>(Z, spec0 + (size_t)plane * N * L, j0, T, N, tw);
}

}  // namespace admm
