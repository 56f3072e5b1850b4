// plane_iso.hip -- the isotropic (BT) solve of 256 x 256 planes with the line spectra resident in the CU
// (included by plane_launch.hip after plane_kernel.hip; same lane-pair / column-buffer machinery).
//
// BT couples every plane of the batch through the per-pixel norm |s|(i,j) = sqrt(sum over planes and both
// channels of s^2) (/root/reference/src/ops/ops.jl:6,10), so an iteration cannot finish inside one
// workgroup: the prox needs the whole batch's s_k first.  Each iteration is therefore split at that point
// into two launches instead of a grid-wide barrier (no co-residency requirement, so the branches of a
// Parallel and other streams can share the GPU freely):
//   plane256_iso_kernel(k)   one workgroup per plane:
//       k > 0:  B phase  s_k, f_k -> w = z - u = f s - (s - f s) -> v = H^T y + rho D^T w     (row_iso_b)
//               line forward
//       column phase (x C: the x-update of ops.jl:86), line inverse -> x_{k+1}
//       A phase  s_{k+1} = D x_{k+1} + (s_k - f_k s_k) stored, q = sum over channels of s_{k+1}^2  (row_iso_a)
//       (k = 0 starts from y: H^T y, line forward; the last launch writes x instead of the A phase)
//   iso_norm_kernel(k+1)     |s_{k+1}| = sqrt(sum over the branch's planes of q), f_{k+1} = max(1 - tau/|s|, 0)
//                            (bt_f; a sharded batch splits it: shard sums, the caller's all-reduce, factor)
// Recording for the reverse sweep (below): s_{k+1} goes to trajectory slot k instead of in place, and
// |s_{k+1}| to norm slot k.
// Every per-pixel map is lane-native like s (element (register n, thread t) at [n][t], float2 = the
// lane's pixel pair), so all of it is read and written in whole-wave contiguous runs.
// HBM per pixel and iteration: B phase s_k 8 + H^T y 4, A phase s_k 8 + s_{k+1} 8 + q 4, norm q 4 (f, the
// branch's 256 KiB map, is L2-resident): 36 B, against 44 and four launches for the 2-pass step
// (column, iso_a, iso_r, iso_b) with the spectrum through HBM twice.

namespace admm {
namespace plane {

// registers of s / map loads in flight ahead of the one being processed in the iso row phases
#ifndef ISO_PD
#define ISO_PD 2
#endif


// BT factor f = max(1 - tau/n, 0) from r = rcp(n) (v_rcp_f32: one rounding off the quotient, the same
// expression in the forward's iso_norm_kernel and the reverse sweep, so the sweep re-forms f bit for bit;
// n = 0 gives -inf -> 0, and 0/0 NaN is kept as the reference's max(NaN, 0) does, ops.jl:10)
__device__ __forceinline__ float bt_f(float tau, float r) {
    const float f = 1.0f - tau * r;
    return f != f ? f : fmaxf(f, 0.0f);
}

// A phase: x (registers 0..31, staged 32..63 in the column buffer) -> s_{k+1} = D x + u_k, u_k = s_k - f_k s_k
// (first: u = 0), stored to sst (may alias sld: every thread reads its own elements before writing them);
// q = (s1^2 + s2^2 of the lane's two pixels) to qst.  Neighbours as in row_update.
__device__ __forceinline__ void row_iso_a(float2 (&S)[64], rsrc_t sld, rsrc_t sst, rsrc_t fld, rsrc_t qst, float2* xb,
                                          float2* colbuf, int t, bool hb, bool first) {
    (void)first;
    constexpr int PD = ISO_PD, NR = PD + 1;
    const int lane = t & 63, w = t >> 6;
    const bool top = lane < 2, bot = lane >= 62;
    float2* stg = colbuf + t;
    float2* stg2 = stg + 16 * kPT;
    if (bot) {
#pragma unroll
        for (int n = 0; n < 32; ++n) xb[(w * 2 + hb) * 64 + n] = S[n];
#pragma unroll
        for (int m = 0; m < 16; ++m) xb[(w * 2 + hb) * 64 + 32 + m] = stg[m * kPT];
#pragma unroll
        for (int m = 0; m < 16; ++m) xb[(w * 2 + hb) * 64 + 48 + m] = stg2[m * kPT];
    }
    const float x63y = stg2[15 * kPT].y;
    lds_barrier();
    sched_fence();
    float4 sr[NR];
    float2 fr[NR];
#pragma unroll
    for (int i = 0; i < PD; ++i) {
        sr[i] = bld4(sld, t * 16, i * kPT * 16);
        fr[i] = bld2(fld, t * 8, i * kPT * 8);
    }
    const float2* xbp = xb + (((w + 7) & 7) * 2 + hb) * 64;   // previous wave's last line
#pragma unroll
    for (int n = 0; n < 64; ++n) {
        if (n + PD < 64) {
            const int q = (n + PD) % NR;
            __asm__ volatile("" ::"v"(sr[q].x), "v"(sr[q].y), "v"(sr[q].z), "v"(sr[q].w), "v"(fr[q].x), "v"(fr[q].y));
            sr[q] = bld4(sld, t * 16, (n + PD) * kPT * 16);
            fr[q] = bld2(fld, t * 8, (n + PD) * kPT * 8);
        }
        if (n == 32) {   // x of registers 32..63 back from the staging slots (x[31] is still in S[31])
#pragma unroll
            for (int m = 0; m < 16; ++m) S[32 + m] = stg[m * kPT];
#pragma unroll
            for (int m = 0; m < 16; ++m) S[48 + m] = stg2[m * kPT];
            sched_fence();
        }
        float2 x = S[n];
        const float xl = swapf(hb ? (n == 0 ? x63y : S[(n + 63) & 63].y) : x.y);   // pixel before the lane's first
        const float2 xub = xbp[n];
        float2 xu = make_float2(lane_up2(x.x), lane_up2(x.y));   // line r-1
        xu.x = top ? xub.x : xu.x;
        xu.y = top ? xub.y : xu.y;
        const float4 a = sr[n % NR];
        const float2 f = fr[n % NR];
        // u_k = s_k - f s_k (z = f s, ops.jl:10), channel pairs (x, z) at pixel p and (y, w) at p + 1
        // (first: sld and fld are resources of size 0, so a = f = 0 and u = 0 without a select)
        float4 u = make_float4(a.x - f.x * a.x, a.y - f.y * a.y, a.z - f.x * a.z, a.w - f.y * a.w);
        if (first) u = make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 s = make_float4((x.x - xu.x) + u.x, (x.y - xu.y) + u.y, (x.x - xl) + u.z, (x.y - x.x) + u.w);
        bst4(sst, t * 16, n * kPT * 16, s);
        bst2(qst, t * 8, n * kPT * 8, make_float2(s.x * s.x + s.z * s.z, s.y * s.y + s.w * s.w));
        sched_fence();
    }
}

// B phase: S <- v = H^T y + rho D^T w, w = z - u = f s - (s - f s) of s_k (sld), f_k (fld), H^T y (hp).
// The D^T neighbours as in row_update (register n+1 / partner lane / line r+1, the next wave's first line
// through the wb buffer after the barrier).
__device__ __forceinline__ void row_iso_b(float2 (&S)[64], rsrc_t sld, rsrc_t fld, rsrc_t hp, float2* wb, float2* sink,
                                          int t, bool hb, float rho) {
    constexpr int PD = ISO_PD, NR = PD + 1;
    const int lane = t & 63, w = t >> 6;
    const bool top = lane < 2, bot = lane >= 62;
    float4 sr[NR];
    float2 fr[NR], hr[NR];
#pragma unroll
    for (int i = 0; i < PD; ++i) {
        sr[i] = bld4(sld, t * 16, i * kPT * 16);
        fr[i] = bld2(fld, t * 8, i * kPT * 8);
        hr[i] = bld2(hp, t * 8, i * kPT * 8);
    }
    float2* wbm = top ? wb + (w * 2 + hb) * 64 : sink + w * 128 + lane;
    float4 wc[2];
    float2 hc[2];
    float w2x0 = 0.0f;
#pragma unroll
    for (int n = 0; n < 64; ++n) {
        if (n + PD < 64) {
            const int q = (n + PD) % NR;
            __asm__ volatile("" ::"v"(sr[q].x), "v"(sr[q].y), "v"(sr[q].z), "v"(sr[q].w), "v"(fr[q].x), "v"(fr[q].y),
                             "v"(hr[q].x), "v"(hr[q].y));
            sr[q] = bld4(sld, t * 16, (n + PD) * kPT * 16);
            fr[q] = bld2(fld, t * 8, (n + PD) * kPT * 8);
            hr[q] = bld2(hp, t * 8, (n + PD) * kPT * 8);
        }
        const float4 a = sr[n % NR];
        const float2 f = fr[n % NR];
        const float4 wv = make_float4(f.x * a.x - (a.x - f.x * a.x), f.y * a.y - (a.y - f.y * a.y),
                                      f.x * a.z - (a.z - f.x * a.z), f.y * a.w - (a.w - f.y * a.w));
        wbm[n] = make_float2(wv.x, wv.y);
        if (n == 0) {
            w2x0 = wv.z;
        } else {
            S[n - 1] = finalize(wc[(n - 1) & 1], wv, hc[(n - 1) & 1], hb, bot, rho);
        }
        wc[n & 1] = wv;
        hc[n & 1] = hr[n % NR];
        sched_fence();
    }
    S[63] = finalize(wc[1], make_float4(0.f, 0.f, w2x0, 0.f), hc[1], hb, bot, rho);
    lds_barrier();
    if (bot) {
        const float2* wbn = wb + (((w + 1) & 7) * 2 + hb) * 64;   // next wave's first line
#pragma unroll
        for (int n = 0; n < 64; ++n) {
            const float2 a = wbn[n];
            S[n].x = fmaf(-rho, a.x, S[n].x);
            S[n].y = fmaf(-rho, a.y, S[n].y);
        }
    }
}

// One iteration k = 0 .. K-1 of the isotropic solve (see the file header).  grid = planes (x Branches),
// block 512, dynamic LDS kLdsBytes.  s_in / s_out: lane-native s_k (k > 0) / s_{k+1} (the same state buffer, or
// consecutive trajectory slots when the solve is recorded for the adjoint); fmap: the branch's f_k (k > 0);
// qpart: per plane q of s_{k+1} (k + 1 < K).
template <bool PSF>
__global__ __launch_bounds__(kPT) void plane256_iso_kernel(const float* __restrict__ y, float* __restrict__ x_out,
                                                           const float* __restrict__ Cf, const float* __restrict__ C0b,
                                                           const float2* __restrict__ Gf, const float2* __restrict__ G0b,
                                                           float2* __restrict__ hln,
                                                           // s_in == s_out (in place) when no trajectory is
                                                           // recorded, so neither is __restrict__
                                                           const float4* s_in, float4* s_out,
                                                           const float2* __restrict__ fmap,
                                                           float2* __restrict__ qpart, const float* __restrict__ prm,
                                                           int k, int K, Branches br) {
    const BranchOf bo = branch_of(br, blockIdx.x);
    Cf += (size_t)bo.i * br.tab_f;
    C0b += (size_t)bo.i * br.tab_f;
    Gf = reinterpret_cast<const float2*>(reinterpret_cast<const float*>(Gf) + (size_t)bo.i * br.tab_f);
    G0b = reinterpret_cast<const float2*>(reinterpret_cast<const float*>(G0b) + (size_t)bo.i * br.tab_f);
    prm += (size_t)bo.i * br.prm_f;
    fmap += (size_t)bo.i * 64 * kPT;
    const float rho = prm[1];
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float2* colbuf = reinterpret_cast<float2*>(smem_raw);
    float2* tw = colbuf + kColF2;
    float2* xb = tw + kTwF2;
    float2* wb = xb + kBndF2;
    float2* sink = wb + kBndF2;
    float2* mir = sink;
    const int t = threadIdx.x;
    float* c0l = reinterpret_cast<float*>(sink + kDumF2);
    if (t < 256) c0l[t] = C0b[t];
    const bool hb = t & 1;
    const int r = t >> 1;
    const size_t plane = blockIdx.x;
    if (t < 256) {
        const int q = t >> 5, kk = t & 31;
        double sn, cs;
        sincospi((double)(q * kk) / 128.0, &sn, &cs);
        tw[q * kTQ + kk] = make_float2((float)cs, (float)-sn);
    }
    constexpr unsigned kS4 = 64 * kPT * 16, kS2 = 64 * kPT * 8;
    const rsrc_t hp = make_rsrc(hln + plane * kHtyStrideF2, kS2);
    const rsrc_t sp = make_rsrc(s_in + plane * 64 * kPT, kS4);        // s_k (k > 0)
    const rsrc_t so = make_rsrc(s_out + plane * 64 * kPT, kS4);       // s_{k+1}: in place, or the next trajectory slot
    const rsrc_t fp = make_rsrc(fmap, kS2);
    const rsrc_t cfr = make_rsrc(Cf, kTab * 4);
    const rsrc_t gfr = make_rsrc(Gf, PSF ? kTab * 8 : 0);
    float2 S[64];
    if (k == 0) {
        const float2* yrow = reinterpret_cast<const float2*>(y + bo.in_plane * 65536 + (size_t)r * 256);
#pragma unroll
        for (int n = 0; n < 64; ++n) S[n] = yrow[2 * n + hb];
        if constexpr (PSF) {
            line_forward_pair(S, hb);
            pin_regs(S);
            column_phase<1>(S, colbuf, tw, mir, cfr, C0b, gfr, G0b, t, hb);
            line_inverse_pair_staged(S, hb, colbuf + t, colbuf + t + 16 * kPT);
#pragma unroll
            for (int m = 0; m < 32; ++m) S[32 + m] = colbuf[t + m * kPT];
        }
#pragma unroll
        for (int n = 0; n < 64; ++n) bst2(hp, t * 8, n * kPT * 8, S[n]);
        // the c0l / twiddle writes above are made visible by the column phase's first barrier
    } else {
        lds_barrier();   // c0l / twiddles written above; the B phase's wb exchange has its own barrier
        row_iso_b(S, sp, fp, hp, wb, sink, t, hb, rho);
    }
    line_forward_pair(S, hb);
    pin_regs(S);
    column_half<0, 0>(S, colbuf, tw, mir, cfr, c0l, gfr, G0b, t, hb);
    column_half<0, 1>(S, colbuf, tw, mir, cfr, c0l, gfr, G0b, t, hb);
    line_inverse_pair_staged(S, hb, colbuf + t, colbuf + t + 16 * kPT);
    if (k + 1 == K) {
#pragma unroll
        for (int m = 0; m < 16; ++m) S[32 + m] = colbuf[t + m * kPT];
#pragma unroll
        for (int m = 0; m < 16; ++m) S[48 + m] = colbuf[t + (16 + m) * kPT];
        float2* xrow = reinterpret_cast<float2*>(x_out + bo.out_plane * 65536 + (size_t)r * 256);
#pragma unroll
        for (int n = 0; n < 64; ++n) xrow[2 * n + hb] = S[n];
        return;
    }
    const rsrc_t none = make_rsrc(s_out, 0);
    const rsrc_t qst = make_rsrc(qpart + plane * 64 * kPT, kS2);
    row_iso_a(S, k == 0 ? none : sp, so, k == 0 ? none : fp, qst, xb, colbuf, t, hb, k == 0);
}

// |s|^2 of every pixel summed over one branch's planes (fixed order: slice j of 4 adds planes j, j+4, ...,
// the slices then in order: deterministic), f = max(1 - tau/|s|, 0) (ops.jl:10; NaN kept as the
// reference's 0/0 gives it).  grid (64 * 512 / 64, nbr) x 256: 64 lane-native float2 elements per block.
// Sharded batch (admm_batch_reducer): sum_out != NULL writes this shard's sums there and stops; after the
// caller's all-reduce of that map, sum_in != NULL takes the sums from it instead of the planes.
__global__ __launch_bounds__(256) void iso_norm_kernel(const float2* __restrict__ qpart, float2* __restrict__ fmap,
                                                       float2* __restrict__ nrm_out, const float* __restrict__ prm,
                                                       Branches br, float2* __restrict__ sum_out,
                                                       const float2* __restrict__ sum_in) {
    __shared__ float2 red[256];
    const int i = blockIdx.y;
    const int e = blockIdx.x * 64 + (threadIdx.x & 63), slice = threadIdx.x >> 6;
    constexpr size_t kE = 64 * kPT;   // float2 elements per plane
    float sx, sy;
    if (sum_in) {
        if (slice) return;
        const float2 v = sum_in[(size_t)i * kE + e];
        sx = v.x, sy = v.y;
    } else {
        const float2* q = qpart + (size_t)i * br.ppb * kE + e;
        float2 a = make_float2(0.f, 0.f);
#pragma unroll 16   // (16 plane loads in flight per thread: the sums stay in the same order)
        for (int p = slice; p < br.ppb; p += 4) {
            const float2 v = q[(size_t)p * kE];
            a.x += v.x;
            a.y += v.y;
        }
        red[threadIdx.x] = a;
        __syncthreads();
        if (slice) return;
        const float2 b = red[64 + threadIdx.x], c = red[128 + threadIdx.x], d = red[192 + threadIdx.x];
        sx = ((a.x + b.x) + c.x) + d.x, sy = ((a.y + b.y) + c.y) + d.y;
        if (sum_out) {
            sum_out[(size_t)i * kE + e] = make_float2(sx, sy);
            return;
        }
    }
    const float tau = prm[(size_t)i * br.prm_f];
    const float nx = sqrtf(sx), ny = sqrtf(sy);
    fmap[(size_t)i * kE + e] = make_float2(bt_f(tau, __builtin_amdgcn_rcpf(nx)), bt_f(tau, __builtin_amdgcn_rcpf(ny)));
    if (nrm_out) nrm_out[(size_t)i * kE + e] = make_float2(nx, ny);
}


// =============================================================================================
// Isotropic ADJOINT at 256 x 256 (reverse sweep of the above; tests/kernel_model.py tvd_model_grads(iso=True)
// states it, admm_backward.hip iso_adj_* is the 2-pass form).  With f = max(1 - tau/n, 0) and n = |s_{k-1}|
// (the recorded batch norm), reverse step k = K .. 1:
//   vbar_k = A^-1 g_k (g_K = x_bar, else D^T sbar_k),  wbar = rho D vbar_k,
//   R = sum over planes and channels of s_{k-1} (2 wbar - sbar_k)                      (batch map, k >= 2)
//   sbar_{k-1} = (2f - 1) wbar + (1 - f) sbar_k + [n > tau] (tau / n^3) R s_{k-1},  tau_bar += sum [n > tau] (-R / n)
// split like the forward at the batch sum:
//   plane256_isoadj_kernel(k)  B phase of step k+1 (k < K: vbar_{k+1} saved, s_k, sbar_{k+1}, R_{k+1}, n_k ->
//                              sbar_k stored, S = g_k = D^T sbar_k), line forward, column phase, line inverse ->
//                              vbar_k; A phase (vbar_k saved, Vsum += vbar_k, R partial of s_{k-1}, sbar_k)
//   iso_radj_kernel(k)         R_k = sum over the branch's planes, tau_bar partials (k >= 2)
// No rho_bar (its <D vbar, D x_k> would need D x_k, i.e. s_k and u_{k-1}: the 2-pass iso sweep keeps it).
// HBM per pixel and step: B: vbar 4, s_k 8, sbar in 8 / out 8; A: vbar out 4, s_{k-1} 8, sbar_k 8, R partial 4;
// the R sum 4 (Vsum in / out 8 more when y_bar is wanted): 56 B, against 72 and four launches (2-pass).
// =============================================================================================

// A phase of reverse step k: v = vbar_k (registers 0..31, 32..63 staged).  Saves vbar_k (vst), accumulates
// Vsum (WV: vlr in, vsr out at vso + n vss -- the natural layout on the last step), and with R (k >= 2) writes
// the plane's R partial sum_ch s_{k-1} (2 wbar - sbar_k) (s1p, sbl in; rst out).
template <bool WV>
__device__ __forceinline__ void row_isoadj_a(float2 (&S)[64], rsrc_t vst, rsrc_t vlr, rsrc_t vsr, unsigned vso,
                                             unsigned vss, rsrc_t s1p, rsrc_t sbl, rsrc_t rst, float2* xb, float2* colbuf,
                                             int t, bool hb, float rho) {
    constexpr int PD = ISO_PD, NR = PD + 1;
    const int lane = t & 63, w = t >> 6;
    const bool top = lane < 2, bot = lane >= 62;
    float2* stg = colbuf + t;
    float2* stg2 = stg + 16 * kPT;
    if (bot) {
#pragma unroll
        for (int n = 0; n < 32; ++n) xb[(w * 2 + hb) * 64 + n] = S[n];
#pragma unroll
        for (int m = 0; m < 16; ++m) xb[(w * 2 + hb) * 64 + 32 + m] = stg[m * kPT];
#pragma unroll
        for (int m = 0; m < 16; ++m) xb[(w * 2 + hb) * 64 + 48 + m] = stg2[m * kPT];
    }
    const float v63y = stg2[15 * kPT].y;
    lds_barrier();
    sched_fence();
    float4 s1r[NR], sbr[NR];
    float2 vr[NR];
#pragma unroll
    for (int i = 0; i < PD; ++i) {
        s1r[i] = bld4(s1p, t * 16, i * kPT * 16);
        sbr[i] = bld4(sbl, t * 16, i * kPT * 16);
        if constexpr (WV) vr[i] = bld2(vlr, t * 8, i * kPT * 8);
    }
    const float2* xbp = xb + (((w + 7) & 7) * 2 + hb) * 64;
#pragma unroll
    for (int n = 0; n < 64; ++n) {
        if (n + PD < 64) {
            const int q = (n + PD) % NR;
            __asm__ volatile("" ::"v"(s1r[q].x), "v"(s1r[q].y), "v"(s1r[q].z), "v"(s1r[q].w), "v"(sbr[q].x),
                             "v"(sbr[q].y), "v"(sbr[q].z), "v"(sbr[q].w));
            s1r[q] = bld4(s1p, t * 16, (n + PD) * kPT * 16);
            sbr[q] = bld4(sbl, t * 16, (n + PD) * kPT * 16);
            if constexpr (WV) vr[q] = bld2(vlr, t * 8, (n + PD) * kPT * 8);
        }
        if (n == 32) {
#pragma unroll
            for (int m = 0; m < 16; ++m) S[32 + m] = stg[m * kPT];
#pragma unroll
            for (int m = 0; m < 16; ++m) S[48 + m] = stg2[m * kPT];
            sched_fence();
        }
        float2 v = S[n];
        const float vl = swapf(hb ? (n == 0 ? v63y : S[(n + 63) & 63].y) : v.y);
        const float2 vub = xbp[n];
        float2 vu = make_float2(lane_up2(v.x), lane_up2(v.y));
        vu.x = top ? vub.x : vu.x;
        vu.y = top ? vub.y : vu.y;
        bst2(vst, t * 8, n * kPT * 8, v);
        if constexpr (WV) {
            const float2 vo = vr[n % NR];
            bst2(vsr, vso, n * vss, make_float2(vo.x + v.x, vo.y + v.y));
        }
        const float4 a = s1r[n % NR], b = sbr[n % NR];
        const float w0 = rho * (v.x - vu.x), w1 = rho * (v.y - vu.y), w2 = rho * (v.x - vl), w3 = rho * (v.y - v.x);
        const float r0 = a.x * (2.0f * w0 - b.x) + a.z * (2.0f * w2 - b.z);
        const float r1 = a.y * (2.0f * w1 - b.y) + a.w * (2.0f * w3 - b.w);
        bst2(rst, t * 8, n * kPT * 8, make_float2(r0, r1));
        sched_fence();
    }
}

// B phase of reverse step k+1 (producing sbar_k and g_k = D^T sbar_k): vbar_{k+1} in S[0..31] and in the
// staging slots (registers 32..63), the register plan of row_adjoint (plane_kernel.hip): at the half-way point
// the slots swap vbar[32..63] in and g[0..30] out.  s1p: s_k; sbl: sbar_{k+1} (in) and sbs: sbar_k (out, the
// same state in place); rp: R_{k+1}; np: n_k = |s_k|.
__device__ __forceinline__ void row_isoadj_b(float2 (&S)[64], rsrc_t s1p, rsrc_t sbl, rsrc_t sbs, rsrc_t rp, rsrc_t np,
                                             float2* xb, float2* wb, float2* sink, float2* colbuf, int t, bool hb,
                                             float tau, float rho) {
    constexpr int PD = ISO_PD, NR = PD + 1;
    const int lane = t & 63, w = t >> 6;
    const bool top = lane < 2, bot = lane >= 62;
    float2* stg = colbuf + t;
    float2* stg2 = stg + 16 * kPT;
    if (bot) {
#pragma unroll
        for (int n = 0; n < 32; ++n) xb[(w * 2 + hb) * 64 + n] = S[n];
#pragma unroll
        for (int m = 0; m < 16; ++m) xb[(w * 2 + hb) * 64 + 32 + m] = stg[m * kPT];
#pragma unroll
        for (int m = 0; m < 16; ++m) xb[(w * 2 + hb) * 64 + 48 + m] = stg2[m * kPT];
    }
    const float v63y = stg2[15 * kPT].y;
    lds_barrier();
    sched_fence();
    float4 s1r[NR], sbr[NR];
    float2 rr[NR], nr[NR];
#pragma unroll
    for (int i = 0; i < PD; ++i) {
        s1r[i] = bld4(s1p, t * 16, i * kPT * 16);
        sbr[i] = bld4(sbl, t * 16, i * kPT * 16);
        rr[i] = bld2(rp, t * 8, i * kPT * 8);
        nr[i] = bld2(np, t * 8, i * kPT * 8);
    }
    const float2* xbp = xb + (((w + 7) & 7) * 2 + hb) * 64;
    float2* wbm = top ? wb + (w * 2 + hb) * 64 : sink + w * 128 + lane;
    float4 wc[2];
    float w2x0 = 0.0f;
    const float2 zero2 = make_float2(0.0f, 0.0f);
#pragma unroll
    for (int n = 0; n < 64; ++n) {
        if (n + PD < 64) {
            const int q = (n + PD) % NR;
            __asm__ volatile("" ::"v"(s1r[q].x), "v"(s1r[q].y), "v"(s1r[q].z), "v"(s1r[q].w), "v"(sbr[q].x),
                             "v"(sbr[q].y), "v"(sbr[q].z), "v"(sbr[q].w), "v"(rr[q].x), "v"(rr[q].y), "v"(nr[q].x),
                             "v"(nr[q].y));
            s1r[q] = bld4(s1p, t * 16, (n + PD) * kPT * 16);
            sbr[q] = bld4(sbl, t * 16, (n + PD) * kPT * 16);
            rr[q] = bld2(rp, t * 8, (n + PD) * kPT * 8);
            nr[q] = bld2(np, t * 8, (n + PD) * kPT * 8);
        }
        if (n == 32) {   // half-way: vbar[32..63] in, g[0..30] out (vbar[31] still pending in S[31])
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                const float2 xv = stg[m * kPT];
                stg[m * kPT] = S[m];
                S[32 + m] = xv;
            }
#pragma unroll
            for (int m = 0; m < 15; ++m) {
                const float2 xv = stg2[m * kPT];
                stg2[m * kPT] = S[16 + m];
                S[48 + m] = xv;
            }
            S[63] = stg2[15 * kPT];
            sched_fence();
        }
        float2 v = S[n];
        const float vl = swapf(hb ? (n == 0 ? v63y : S[(n + 63) & 63].y) : v.y);
        const float2 vub = xbp[n];
        float2 vu = make_float2(lane_up2(v.x), lane_up2(v.y));
        vu.x = top ? vub.x : vu.x;
        vu.y = top ? vub.y : vu.y;
        const float4 a = s1r[n % NR], b = sbr[n % NR];
        const float2 R = rr[n % NR], nn = nr[n % NR];
        // per pixel (p: x / z channels, p + 1: y / w): f = max(1 - tau/n, 0), c = [n > tau] (tau / n^3) R
        const float r0 = __builtin_amdgcn_rcpf(nn.x), r1 = __builtin_amdgcn_rcpf(nn.y);
        const float f0 = bt_f(tau, r0), f1 = bt_f(tau, r1);
        const float c0 = nn.x > tau ? tau * (r0 * r0 * r0) * R.x : 0.0f;
        const float c1 = nn.y > tau ? tau * (r1 * r1 * r1) * R.y : 0.0f;
        const float w0 = rho * (v.x - vu.x), w1 = rho * (v.y - vu.y), w2 = rho * (v.x - vl), w3 = rho * (v.y - v.x);
        const float4 nb = make_float4((2.0f * f0 - 1.0f) * w0 + (1.0f - f0) * b.x + c0 * a.x,
                                      (2.0f * f1 - 1.0f) * w1 + (1.0f - f1) * b.y + c1 * a.y,
                                      (2.0f * f0 - 1.0f) * w2 + (1.0f - f0) * b.z + c0 * a.z,
                                      (2.0f * f1 - 1.0f) * w3 + (1.0f - f1) * b.w + c1 * a.w);
        bst4(sbs, t * 16, n * kPT * 16, nb);
        wbm[n] = make_float2(nb.x, nb.y);
        if (n == 0) {
            w2x0 = nb.z;
        } else {
            S[n - 1] = finalize(wc[(n - 1) & 1], nb, zero2, hb, bot, 1.0f);
        }
        wc[n & 1] = nb;
        sched_fence();
    }
    S[63] = finalize(wc[1], make_float4(0.f, 0.f, w2x0, 0.f), zero2, hb, bot, 1.0f);
#pragma unroll
    for (int m = 0; m < 16; ++m) S[m] = stg[m * kPT];
#pragma unroll
    for (int m = 0; m < 15; ++m) S[16 + m] = stg2[m * kPT];
    lds_barrier();
    if (bot) {
        const float2* wbn = wb + (((w + 1) & 7) * 2 + hb) * 64;   // next wave's first line
#pragma unroll
        for (int n = 0; n < 64; ++n) {
            const float2 a = wbn[n];
            S[n].x -= a.x;
            S[n].y -= a.y;
        }
    }
}

// Reverse step k (K .. 1) of every plane.  xbar: natural layout (k = K), in the chcat layout of Branches;
// traj: s_1..s_{K-1} (slot j = s_{j+1}, slot stride tslot float4); nrm: the branches' |s_k| maps (slot j = n_{j+1},
// per branch 64 x 512 float2, slot stride nslot float2); vbuf: vbar (lane-native, per plane); sbar: state;
// Rmap: the branches' R_{k+1} (k < K); rpart: per plane R partial of step k (k >= 2); WV: Vsum in vsl
// (lane-native), written to vout (natural, per grid plane) on the last step.
template <bool WV>
__global__ __launch_bounds__(kPT) void plane256_isoadj_kernel(const float* __restrict__ xbar, const float* __restrict__ Cf,
                                                              const float* __restrict__ C0b, const float4* __restrict__ traj,
                                                              size_t tslot, const float2* __restrict__ nrm, size_t nslot,
                                                              float2* __restrict__ vbuf, float4* __restrict__ sbar,
                                                              const float2* __restrict__ Rmap, float2* __restrict__ rpart,
                                                              float2* __restrict__ vsl, float* __restrict__ vout,
                                                              const float* __restrict__ prm, int k, int K, Branches br) {
    const BranchOf bo = branch_of(br, blockIdx.x);
    Cf += (size_t)bo.i * br.tab_f;
    C0b += (size_t)bo.i * br.tab_f;
    prm += (size_t)bo.i * br.prm_f;
    const float tau = prm[0], rho = prm[1];
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float2* colbuf = reinterpret_cast<float2*>(smem_raw);
    float2* tw = colbuf + kColF2;
    float2* xb = tw + kTwF2;
    float2* wb = xb + kBndF2;
    float2* sink = wb + kBndF2;
    float2* mir = sink;
    const int t = threadIdx.x;
    float* c0l = reinterpret_cast<float*>(sink + kDumF2);
    if (t < 256) c0l[t] = C0b[t];
    const bool hb = t & 1;
    const int r = t >> 1;
    const size_t plane = blockIdx.x;
    if (t < 256) {
        const int q = t >> 5, kk = t & 31;
        double sn, cs;
        sincospi((double)(q * kk) / 128.0, &sn, &cs);
        tw[q * kTQ + kk] = make_float2((float)cs, (float)-sn);
    }
    constexpr unsigned kS4 = 64 * kPT * 16, kS2 = 64 * kPT * 8;
    constexpr size_t kE = 64 * kPT;
    const rsrc_t cfr = make_rsrc(Cf, kTab * 4);
    const rsrc_t none = make_rsrc(Cf, 0);
    const rsrc_t vbp = make_rsrc(vbuf + plane * kE, kS2);
    const rsrc_t sbp = make_rsrc(sbar + plane * kE, kS4);
    const float4* tb = traj + plane * kE;
    const float2* nb = nrm + (size_t)bo.i * kE;
    float2 S[64];
    if (k == K) {
        const float2* grow = reinterpret_cast<const float2*>(xbar + bo.out_plane * 65536 + (size_t)r * 256);
#pragma unroll
        for (int n = 0; n < 64; ++n) S[n] = grow[2 * n + hb];
        pin_regs(S);
    } else {
        // vbar_{k+1}: registers 0..31 in S, 32..63 in the staging slots (row_isoadj_b)
#pragma unroll
        for (int n = 0; n < 32; ++n) S[n] = bld2(vbp, t * 8, n * kPT * 8);
#pragma unroll
        for (int m = 0; m < 32; ++m) colbuf[t + m * kPT] = bld2(vbp, t * 8, (32 + m) * kPT * 8);
        // B phase of step k+1: s_k = slot k-1, n_k = slot k-1, R_{k+1}
        row_isoadj_b(S, make_rsrc(tb + (size_t)(k - 1) * tslot, kS4), k + 1 < K ? sbp : none, sbp,
                     make_rsrc(Rmap + (size_t)bo.i * kE, kS2), make_rsrc(nb + (size_t)(k - 1) * nslot, kS2), xb, wb,
                     sink, colbuf, t, hb, tau, rho);
        pin_regs(S);
    }
    line_forward_pair(S, hb);
    pin_regs(S);
    column_half<0, 0>(S, colbuf, tw, mir, cfr, c0l, none, nullptr, t, hb);
    column_half<0, 1>(S, colbuf, tw, mir, cfr, c0l, none, nullptr, t, hb);
    line_inverse_pair_staged(S, hb, colbuf + t, colbuf + t + 16 * kPT);
    // A phase of step k: vbar_k saved; Vsum (natural layout into vout on the last step); R partial (k >= 2)
    const rsrc_t vlr = (WV && k < K) ? make_rsrc(vsl + plane * kE, kS2) : none;
    const rsrc_t vsr = !WV ? none : k >= 2 ? make_rsrc(vsl + plane * kE, kS2) : make_rsrc(vout + plane * 65536, 65536 * 4);
    const unsigned vso = k >= 2 ? (unsigned)t * 8 : (unsigned)(r * 1024 + hb * 8);
    const unsigned vss = k >= 2 ? kPT * 8 : 16;
    const rsrc_t s1p = k >= 2 ? make_rsrc(tb + (size_t)(k - 2) * tslot, kS4) : none;
    const rsrc_t sbl = (k >= 2 && k < K) ? sbp : none;
    const rsrc_t rst = k >= 2 ? make_rsrc(rpart + plane * kE, kS2) : none;
    row_isoadj_a<WV>(S, k >= 2 ? vbp : none, vlr, vsr, vso, vss, s1p, sbl, rst, xb, colbuf, t, hb, rho);
}

// R_k of every pixel, summed over one branch's planes (fixed order as iso_norm_kernel), and the step's tau_bar
// partial sum over this block's pixels of [n_{k-1} > tau] (-R / n_{k-1}) (fp64, fixed order) -> part[2 blk + 1]
// (part[2 blk] = 0: no rho_bar).  grid (512, nbr) x 256; part rows per branch: 512 per step.
__global__ __launch_bounds__(256) void iso_radj_kernel(const float2* __restrict__ rpart, float2* __restrict__ Rmap,
                                                       const float2* __restrict__ nrm1, double* __restrict__ part,
                                                       size_t part_branch, const float* __restrict__ prm, Branches br) {
    __shared__ float2 red[256];
    const int i = blockIdx.y;
    const int e = blockIdx.x * 64 + (threadIdx.x & 63), slice = threadIdx.x >> 6;
    constexpr size_t kE = 64 * kPT;
    const float2* q = rpart + (size_t)i * br.ppb * kE + e;
    float2 a = make_float2(0.f, 0.f);
#pragma unroll 16
    for (int p = slice; p < br.ppb; p += 4) {
        const float2 v = q[(size_t)p * kE];
        a.x += v.x;
        a.y += v.y;
    }
    red[threadIdx.x] = a;
    __syncthreads();
    double tb = 0.0;
    if (slice == 0) {
        const float2 b = red[64 + threadIdx.x], c = red[128 + threadIdx.x], d = red[192 + threadIdx.x];
        const float Rx = ((a.x + b.x) + c.x) + d.x, Ry = ((a.y + b.y) + c.y) + d.y;
        Rmap[(size_t)i * kE + e] = make_float2(Rx, Ry);
        const float tau = prm[(size_t)i * br.prm_f];
        const float2 nn = nrm1[(size_t)i * kE + e];
        tb = (nn.x > tau ? (double)(-Rx / nn.x) : 0.0) + (nn.y > tau ? (double)(-Ry / nn.y) : 0.0);
        for (int off = 32; off > 0; off >>= 1) tb += __shfl_down(tb, off);
        if (threadIdx.x == 0) {
            part[(size_t)i * part_branch + 2 * blockIdx.x] = 0.0;
            part[(size_t)i * part_branch + 2 * blockIdx.x + 1] = tb;
        }
    }
}
}  // namespace plane
}  // namespace admm
