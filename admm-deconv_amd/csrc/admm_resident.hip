// admm_resident.hip -- the whole K-iteration anisotropic ADMM solve of ONE plane per workgroup for smooth
// non-power-of-two sides <= 256 (reference: tvd_fft_cpu / tvd_fft_gpu, /root/reference/src/ops/ops.jl:46-93 /
// :132-176; any M x N through FFTW / CUFFT plans, ops.jl:26,86).
//
// Why: the smooth 2-pass path (admm_smooth.hip) moves the line spectrum through HBM twice per iteration
// (44 B/px/iter at 250^2: column pass 8, line inverse 8, update 28).  Here the half spectrum never leaves the
// CU: 512 threads hold it in registers (250^2: 126 bins x 250 lines = 63 float2 per thread) and the
// transforms run in LDS, one chunk at a time.  Per iteration the only HBM traffic is the ADMM state
// s = Dx + u (read + write, 8 B/px each) and H^T y (4 B/px): 20 B/px, as in the 256^2 kernel
// (plane_kernel.hip).
//
// Register layout: the H bins are dealt into NCC column chunks of KBC bins; thread t = kk * LS + jt (LS = 512 /
// KBC line slots) holds bin c KBC + kk of every chunk c, lines jt, jt + LS, ...:
// S[c NR + r] = X(line r LS + jt, bin c KBC + kk).  A column chunk is register range c and a line chunk
// (a multiple of LS lines) register range r, so every thread takes part in every phase and no register is
// ever written under a lane condition: a lane-conditional write keeps the old value live next to the new
// one (a phi the register allocator resolves with copies), which at 250^2 cost 288 B/lane of spills.
// Both staging directions are plain LDS accesses at compile-time offsets from a per-thread base.
//
// Per iteration:
//   column phase  per chunk of KBC bins: S -> LDS [bin][line], dim-2 FFT (compile-time Stockham plan,
//                 fft_smooth.hpp), x Ct (C / (MN), ops.jl:86) fused between the last forward and the first
//                 inverse pass, IFFT, LDS -> S.
//   line phase    per chunk of T lines plus the two halo lines either side (T + 2 rows): S -> LDS, paired
//                 real inverse transforms -> x rows; then every wave walks its own rows:
//                 s = D x + clip(s_old) (ops.jl:87-92 with u = clip(s)), w = z - u, v = H^T y + rho D^T w,
//                 s stored, v written over x (a wave's first and last rows only after a block barrier: they
//                 are the rows its neighbours read); paired forward transforms of v -> S.
// H^T y itself (with a PSF: F^-1 conj(Sigma_c) F y, ops.jl:71-81) comes from the 2-pass PREP kernels; the
// first iteration's spectrum is its line rFFT, formed here.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "fft_smooth.hpp"
#include "resident_api.hpp"

namespace admm {
namespace rs {

using sm::dftR;
using sm::SP;

constexpr int kNT = 512;                  // threads per workgroup (8 waves, 2 per SIMD)
#ifndef RS_PD
#define RS_PD 3                           // rows of update loads in flight ahead of the row being computed (2-5 within 1-2 %, 3 best: profiles/r04v_resident_pd.txt)
#endif
#ifndef RS_RAD
// radix cap 25: the 250- and 200-point transforms run as 2 passes ({10, 25}, {20, 10}) instead of 3; at 250^2 x 256
// 92.6k -> 98.9k img/s, 200^2 129k -> 167k, the other compiled shapes keep their plans (profiles/r05_resident_rad25.log)
#define RS_RAD 25
#endif
#ifndef RS_PDI
#define RS_PDI 4                          // the same for the isotropic A / B phases (3: 250^2 iso 3.78 -> 3.93 ms)
#endif
#ifndef RS_PINSEP
#define RS_PINSEP 1
#endif
#ifndef RS_U2MAX
#define RS_U2MAX 10
#endif
#ifndef RS_INPLACE
// the anisotropic update rewrites s in place instead of ping-ponging two buffers: 256 planes at 250^2 re-stream
// 192 MiB per iteration instead of 320, inside the 256 MiB Infinity Cache (DESIGN.md s5 "Round 5, resident")
#define RS_INPLACE 1
#endif
constexpr int kRad = RS_RAD;              // radix cap of every transform
constexpr int kLdsBytes = 160 * 1024;     // gfx950 LDS per CU

constexpr int cdiv(int a, int b) { return (a + b - 1) / b; }
constexpr int imax(int a, int b) { return a > b ? a : b; }
constexpr int imin(int a, int b) { return a < b ? a : b; }

__device__ __forceinline__ float clipf(float s, float tau) { return fminf(fmaxf(s, -tau), tau); }
// w = z - u for z = ST(s, tau), u = s - z  (ops.jl:9, :171-173)
__device__ __forceinline__ float prox_w(float s, float tau) { return fabsf(s) > tau ? s - copysignf(2.0f * tau, s) : -s; }

// Buffer resources for the update's HBM traffic (32-bit offsets: a wave-uniform row offset in an SGPR and
// a per-lane constant pixel offset; out-of-range loads return 0)
using rsrc_t = __amdgpu_buffer_rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float bld1(rsrc_t r, unsigned vo, unsigned so) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
}
__device__ __forceinline__ void bst1(rsrc_t r, unsigned vo, unsigned so, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, vo, so, 0);
}
using u32x2 = unsigned __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float2 bld2(rsrc_t r, unsigned vo, unsigned so) {
    return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, 0));
}
__device__ __forceinline__ void bst2(rsrc_t r, unsigned vo, unsigned so, float2 v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, vo, so, 0);
}
// G neighbouring floats of one lane, moved by one buffer access
template <int G>
struct Vg {
    float v[G];
    static __device__ __forceinline__ Vg load(rsrc_t r, unsigned vo, unsigned so) {
        Vg x;
        if constexpr (G == 2) {
            const float2 f = bld2(r, vo, so);
            x.v[0] = f.x;
            x.v[1] = f.y;
        } else {
            x.v[0] = bld1(r, vo, so);
        }
        return x;
    }
    __device__ __forceinline__ void store(rsrc_t r, unsigned vo, unsigned so) const {
        if constexpr (G == 2) bst2(r, vo, so, make_float2(v[0], v[1]));
        else bst1(r, vo, so, v[0]);
    }
};

// The thread index through an opaque move: values derived from it are recomputed inside the iteration loop
// rather than hoisted out of it (dozens of per-pass start indices and LDS bases would otherwise stay live
// across all K iterations, next to the 126-VGPR spectrum)
__device__ __forceinline__ int tid() {
    int y;
    __asm__ volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"((int)threadIdx.x));
    return y;
}

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

// ---- in-place mixed-radix transforms -------------------------------------------------------------------
// Radices R_0 .. R_{P-1} (fft_smooth.hpp's plan, increasing, <= kRad).  Pass p works on blocks of
// L_p = LEN / (R_0 .. R_{p-1}) points with stride S_p = L_p / R_p.
//   DIF pass (natural order in): load x[base + r S], DFT over r, x W_L^{j m}, store at base + m S;
//   DIT pass: load at base + m S, x W_L^{j m}, DFT over m, store at base + r S  (base = block L + j).
// DIF passes 0 .. P-1 leave frequency k = m_0 + R_0 m_1 + R_0 R_1 m_2 + .. at position
// pos(k) = m_0 S_0 + m_1 S_1 + ..; DIT passes P-1 .. 0 undo them (conjugate kernels: an unnormalised
// inverse).  Every butterfly reads and writes the same R slots, so a pass needs no barrier of its own and
// holds only R complex values per butterfly -- the spectrum's registers stay free.
template <int LEN>
struct Rad {
    using S = SP<LEN, true, kRad>;
    static constexpr int P = S::P;
    static constexpr int r(int p) { return S::pl.r[p]; }
    static constexpr int L(int p) {
        int l = LEN;
        for (int q = 0; q < p; ++q) l /= r(q);
        return l;
    }
    static constexpr int st(int p) { return L(p) / r(p); }   // S_p
    static constexpr int W(int p) {                           // R_0 .. R_{p-1}
        int w = 1;
        for (int q = 0; q < p; ++q) w *= r(q);
        return w;
    }
    // offset of pass p's twiddles in the compact table: pass q holds W_{L_q}^{j m} for j < S_q, m = 1 .. R_q - 1
    // at [j (R_q - 1) + m - 1]; LEN - 1 entries in all (sum of L_q - L_{q+1})
    static constexpr int toff(int p) {
        int o = 0;
        for (int q = 0; q < p; ++q) o += st(q) > 1 ? st(q) * (r(q) - 1) : 0;
        return o;
    }
};

// The compact twiddle table of a LEN-point plan (Rad::toff) from the setup kernel's exp(-2 pi i n / LEN): the
// R - 1 twiddles of a butterfly are neighbours (paired LDS reads at immediate offsets from one base) where the full
// table put them j m LEN / L apart (one address computation and one read each)
template <int LEN>
__device__ __forceinline__ void fill_twiddles(float2* ct, const float2* __restrict__ full, int nthreads) {
    using RD = Rad<LEN>;
    for (int i = threadIdx.x; i < LEN - 1; i += nthreads) {
        float2 w = make_float2(1.0f, 0.0f);
        static_for<0, RD::P>([&](auto ip) {
            constexpr int p = decltype(ip)::value;
            constexpr int R = RD::r(p), S = RD::st(p), TS = LEN / RD::L(p), o0 = RD::toff(p), o1 = RD::toff(p + 1);
            if (S > 1 && i >= o0 && i < o1) {
                const int rr = i - o0, j = rr / (R - 1), m = 1 + rr - j * (R - 1);
                w = full[j * m * TS];
            }
        });
        ct[i] = w;
    }
}

// position of natural index k after the DIF passes
template <int LEN>
__device__ __forceinline__ int dpos(int k) {
    using RD = Rad<LEN>;
    int pos = 0;
    static_for<0, RD::P>([&](auto ip) {
        constexpr int p = decltype(ip)::value;
        constexpr int R = RD::r(p);
        const int q = k / R;
        pos += (k - q * R) * RD::st(p);
        k = q;
    });
    return pos;
}
// frequency of slot b R + m after the DIF passes (b = butterfly of the last pass): kbase(b) + m W_{P-1}
template <int LEN>
__device__ __forceinline__ int dlast(int b) {
    using RD = Rad<LEN>;
    int k = 0;
    static_for<0, RD::P - 1>([&](auto ip) {
        constexpr int p = RD::P - 2 - decltype(ip)::value;   // least significant digit of b first
        constexpr int R = RD::r(p);
        const int q = b / R;
        k += (b - q * R) * RD::W(p);
        b = q;
    });
    return k;
}

// A wave's lanes over one line of MM pixels: GP neighbouring pixels per lane (Geo::GP), QG slices of 64 lanes.
// LDS float offsets (x at dpos order within a pair row) of the lane's pixels and of its first pixel's left
// neighbour; buffer byte offsets of the lane's pixels (+ the slice's immediate); stores of lanes past the line's
// end go beyond the buffer (dropped) and LDS writes are masked.
template <int MM>
struct RowLanes {
    static constexpr int GP = MM > 64 ? 2 : 1, QG = (MM + 64 * GP - 1) / (64 * GP);
    static constexpr unsigned SL = 256 * GP;
    int po[QG][GP], plo[QG];
    unsigned gl, glst;
    int lane;
    __device__ __forceinline__ RowLanes() {
        lane = tid() & 63;
#pragma unroll
        for (int q = 0; q < QG; ++q) {
            const int i0 = GP * (lane + 64 * q) < MM ? GP * (lane + 64 * q) : 0;
#pragma unroll
            for (int g = 0; g < GP; ++g) po[q][g] = 2 * dpos<MM>(i0 + g);
            plo[q] = 2 * dpos<MM>(i0 == 0 ? MM - 1 : i0 - 1);
        }
        gl = 4u * GP * (unsigned)lane;
        glst = GP * (lane + 64 * (QG - 1)) < MM ? gl : 0x80000000u;
    }
    __device__ __forceinline__ bool valid(int q) const { return q < QG - 1 || GP * (lane + 64 * q) < MM; }
    template <int G>
    __device__ __forceinline__ Vg<G> ld(rsrc_t r, int q, unsigned so) const { return Vg<G>::load(r, gl + SL * q, so); }
    template <int G>
    __device__ __forceinline__ void st(rsrc_t r, int q, unsigned so, const Vg<G>& v) const {
        v.store(r, (q < QG - 1 ? gl : glst) + SL * q, so);
    }
    template <int G>
    __device__ __forceinline__ Vg<G> xget(const float* Xf, int rbase, int q) const {
        Vg<G> x;
#pragma unroll
        for (int g = 0; g < G; ++g) x.v[g] = Xf[rbase + po[q][g]];
        return x;
    }
    template <int G>
    __device__ __forceinline__ void put(float* Xf, int q, int rbase, const Vg<G>& v) const {
        if (valid(q)) {
#pragma unroll
            for (int g = 0; g < G; ++g) Xf[rbase + po[q][g]] = v.v[g];
        }
    }
};

template <bool INV>
__device__ __forceinline__ float2 twv(const float2* __restrict__ tw, int e) {
    float2 w = tw[e];
    if (INV) w.y = -w.y;
    return w;
}

// Accessor of cnt transforms: transform f point n at base[f * FS + n]
template <int FS>
struct Acc {
    float2* base;
    __device__ __forceinline__ float2 ld(int f, int n) const { return base[f * FS + n]; }
    __device__ __forceinline__ void st(int f, int n, float2 v) const { base[f * FS + n] = v; }
};

// one in-place pass p over cnt transforms; butterflies dealt to the block's threads two at a time.
// FMAJ: consecutive threads take one transform's consecutive butterflies (lines); else consecutive
// transforms (columns).
template <int LEN, int p, bool DIT, bool INV, bool FMAJ, int FS>
__device__ __forceinline__ void ipass(int cnt, const float2* __restrict__ tw, Acc<FS> a) {
    using RD = Rad<LEN>;
    constexpr int R = RD::r(p), L = RD::L(p), S = L / R, Q = LEN / R;
    const int total = cnt * Q;
    auto where = [&](int idx, int& f, int& base, int& j) {
        int b;
        if (FMAJ) {
            f = idx / Q;
            b = idx - f * Q;
        } else {
            b = idx / cnt;
            f = idx - b * cnt;
        }
        const int blk = b / S;
        j = b - blk * S;
        base = blk * L + j;
    };
    // tw: the compact table (fill_twiddles): this butterfly's R - 1 twiddles are neighbours
    auto fly = [&](float2 (&v)[R], int j) {
        const float2* tp = tw + RD::toff(p) + j * (R - 1);
        if constexpr (DIT && S > 1) {
#pragma unroll
            for (int m = 1; m < R; ++m) v[m] = cmul(v[m], twv<INV>(tp, m - 1));
        }
        dftR<R, INV>(v);
        if constexpr (!DIT && S > 1) {
#pragma unroll
            for (int m = 1; m < R; ++m) v[m] = cmul(v[m], twv<INV>(tp, m - 1));
        }
    };
    // two butterflies in flight for small radices; one for R > 10 (register pressure next to the spectrum)
    constexpr int U = R <= RS_U2MAX ? 2 : 1;
    // not unrolled: with a compile-time trip count the compiler would interleave the butterflies of several
    // iterations (2 U in flight: ~136 VGPRs of butterfly values next to the spectrum, the 250^2 spills)
#pragma unroll 1
    for (int i0 = tid(); i0 < total; i0 += U * kNT) {
        const int i1 = i0 + kNT;
        int f0, b0, j0, f1 = 0, b1 = 0, j1 = 0;
        where(i0, f0, b0, j0);
        const bool two = U == 2 && i1 < total;
        if (two) where(i1, f1, b1, j1);
        float2 v0[R], v1[R];
#pragma unroll
        for (int r = 0; r < R; ++r) v0[r] = a.ld(f0, b0 + r * S);
        if (two) {
#pragma unroll
            for (int r = 0; r < R; ++r) v1[r] = a.ld(f1, b1 + r * S);
        }
        fly(v0, j0);
#pragma unroll
        for (int r = 0; r < R; ++r) a.st(f0, b0 + r * S, v0[r]);
        if (two) {
            fly(v1, j1);
#pragma unroll
            for (int r = 0; r < R; ++r) a.st(f1, b1 + r * S, v1[r]);
        }
    }
}

// DIF passes [p0, p1) / DIT passes (p1 .. p0], a block barrier after each
template <int LEN, int p0, int p1, bool INV, bool FMAJ, int FS>
__device__ __forceinline__ void dif_passes(int cnt, const float2* tw, Acc<FS> a) {
    static_for<p0, p1>([&](auto ip) {
        ipass<LEN, decltype(ip)::value, false, INV, FMAJ, FS>(cnt, tw, a);
        __syncthreads();
    });
}
template <int LEN, int p0, int p1, bool INV, bool FMAJ, int FS>
__device__ __forceinline__ void dit_passes(int cnt, const float2* tw, Acc<FS> a) {
    static_for<p0, p1>([&](auto ip) {
        ipass<LEN, p1 - 1 - (decltype(ip)::value - p0), true, INV, FMAJ, FS>(cnt, tw, a);
        __syncthreads();
    });
}

template <int MM, int NN>
struct Geo {
    static constexpr int H = MM / 2 + 1;           // bins per line
    static constexpr int kBudget = (kLdsBytes - 512) / 8 - MM - NN;   // float2 slots for the main buffer
    // column chunks n: KBC bins each, LS line slots (even: lines 2f, 2f + 1 in neighbouring lanes), NR
    // registers per chunk; the column buffer holds KBC columns of stride FS >= NR LS (odd: neighbouring
    // columns on distinct banks), so the read-back of a register's padding lines stays in its own column
    static constexpr int kbc(int n) { return cdiv(H, n); }
    static constexpr int ls(int n) { return (kNT / kbc(n)) & ~1; }
    static constexpr int nr(int n) { return cdiv(NN, ls(n)); }
    static constexpr int fs(int n) { return (nr(n) * ls(n)) | 1; }
    static constexpr bool fits(int n) { return ls(n) >= 2 && kbc(n) * fs(n) <= kBudget; }
    // fewest chunks whose spectrum takes at most 2 registers more than the fewest possible: every chunk is a
    // round of column passes with its barriers (250^2: 2 chunks of 32 registers, not 3 of 21; 85.0k vs 84.0k
    // img/s, profiles/r04_resident_variants.txt)
    static constexpr int min_regs() {
        int m = 1 << 30;
        for (int n = 1; n <= 8 && n <= H; ++n)
            if (fits(n) && n * nr(n) < m) m = n * nr(n);
        return m;
    }
    static constexpr int ncc() {
        for (int n = 1; n <= 8 && n <= H; ++n)
            if (fits(n) && n * nr(n) <= min_regs() + 2) return n;
        return 0;
    }
#ifdef RS_NCC_FORCE   // experiments: column chunk count forced
    static constexpr int NCC = fits(RS_NCC_FORCE) ? RS_NCC_FORCE : ncc();
#else
    static constexpr int NCC = ncc();              // column chunks
#endif
    static constexpr int KBC = kbc(NCC);           // bins per column chunk
    static constexpr int LS = ls(NCC);             // line slots
    static constexpr int NR = nr(NCC);             // registers per column chunk
    static constexpr int NREG = NCC * NR;          // spectrum registers (float2) per thread
    static constexpr int FS = fs(NCC);
    static constexpr int QN = cdiv(MM, 64);        // pixels per lane and row in the update
    static constexpr int GP = MM > 64 ? 2 : 1;     // neighbouring pixels per lane in the row update
    static constexpr int QG = cdiv(MM, 64 * GP);   // slices of 64 lanes per row
    // line chunks: TL lines (a multiple of LS: whole registers) + a halo pair either side, as complex pairs
    static constexpr int tl(int n) { return cdiv(cdiv(NN, n), LS) * LS; }
    static constexpr int nlc() {
        for (int n = 1; n <= NN; ++n)
            if ((tl(n) / 2 + 2) * MM <= kBudget) return n;
        return 0;
    }
    static constexpr int NLC = nlc();              // line chunks
    static constexpr int TL = tl(NLC);             // lines per line chunk
    static constexpr int BUF = imax(KBC * FS, (TL / 2 + 2) * MM);
    // LDS rows for each wave's first and last row update (interleaved like a line pair: 2 M floats per wave), so
    // that the row step writes every v through one uniform address select instead of holding those two rows in
    // registers under branches (the neighbouring waves read the x they replace until the block barrier).  Only
    // where it fits beside the geometry above (not at 192^2, whose single line chunk fills the LDS).
    static constexpr int SCR = 8 * MM;             // float2 slots
    static constexpr bool kScr = (size_t)(MM + NN + BUF + SCR) * 8 + 512 <= (size_t)kLdsBytes;
    static constexpr size_t lds_bytes() { return (size_t)(MM + NN + BUF + (kScr ? SCR : 0)) * 8; }
    static_assert(MM % 2 == 0 && NN % 2 == 0 && MM <= 256 && NN <= 256, "resident kernel: even M, N <= 256");
    static_assert(NCC >= 1 && NLC >= 1, "resident kernel: shape does not fit one CU");
    static_assert(LS % 2 == 0 && TL % 2 == 0, "line pairs within a lane pair");
    static_assert(Rad<MM>::P >= 2 && Rad<NN>::P >= 2, "plans of >= 2 passes");
};

struct Thr {
    float2* buf;          // main LDS buffer
    const float2* twm;    // LDS twiddles exp(-2 pi i n / M), exp(-2 pi i n / N)
    const float2* twn;
    int kk, jt;           // bin within a column chunk, line slot
    bool act;             // kk < KBC
};
template <int MM, int NN>
__device__ __forceinline__ Thr thr_of(float2* buf, const float2* twm, const float2* twn) {
    using G = Geo<MM, NN>;
    const unsigned t = (unsigned)tid();
    return {buf, twm, twn, (int)(t / G::LS), (int)(t % G::LS), t < (unsigned)(G::KBC * G::LS)};
}

// ---- column phase, chunk C: bins [kc0, kc1) = registers [C NR, C NR + NR) ---------------------------------
// Three parts: the chunk's registers into the column buffer (column_stage<C>), the transforms with x Ct between
// them (column_passes, the chunk given at run time: LDS and Ct only, no spectrum register), and the read-back
// (column_unstage<C>).  column_phase runs the chunks as a loop that is NOT unrolled, so the passes' code exists
// once instead of once per chunk (RS_COLSHARE; at 250^2 the kernel's iteration loop otherwise exceeds the 64 KiB
// instruction cache two CUs share, DESIGN.md s5 "Round 5, resident").
#ifndef RS_COLSHARE
#define RS_COLSHARE 1
#endif
template <int MM, int NN, int C, int NREG>
__device__ __forceinline__ void column_stage(const float2 (&S)[NREG], const Thr& th,
                                             int kc = imin(Geo<MM, NN>::H, (C + 1) * Geo<MM, NN>::KBC) - C * Geo<MM, NN>::KBC) {
    using G = Geo<MM, NN>;
    constexpr int FS = G::FS, NR = G::NR, R0 = C * NR;
    if (th.kk < kc) {   // stores only: the spectrum registers are not written here
        float2* col = th.buf + th.kk * FS;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const int j = r * G::LS + th.jt;
            if (r < NR - 1 || j < NN) col[j] = S[R0 + r];
        }
    }
}
template <int MM, int NN, int C, int NREG>
__device__ __forceinline__ void column_unstage(float2 (&S)[NREG], const Thr& th,
                                               int kc = imin(Geo<MM, NN>::H, (C + 1) * Geo<MM, NN>::KBC) - C * Geo<MM, NN>::KBC) {
    using G = Geo<MM, NN>;
    constexpr int NR = G::NR, R0 = C * NR;
    // every thread reads back every register of the chunk (threads past the chunk's bins: a valid column,
    // values never used; padding lines j >= NN: the column's padding slots, never used either)
    const float2* col = th.buf + imin(th.kk, kc - 1) * G::FS;
#pragma unroll
    for (int r = 0; r < NR; ++r) S[R0 + r] = col[r * G::LS + th.jt];
}
// the staged chunk's bins [kc0, kc0 + kc): dim-2 FFT, x Ct at the slot's frequency, IFFT (barrier before and after)
template <int MM, int NN>
__device__ __forceinline__ void column_passes(int kc0, int kc, const Thr& th, const float* __restrict__ Ct) {
    using G = Geo<MM, NN>;
    using RD = Rad<NN>;
    constexpr int KB = G::KBC, FS = G::FS, H = G::H, P = RD::P;
    __syncthreads();
    const Acc<FS> a{th.buf};
    dif_passes<NN, 0, P - 1, false, false, FS>(KB, th.twn, a);
    // last DIF pass (S = 1: no twiddles) -> x Ct at the slot's frequency -> first DIT pass, in registers
    {
        constexpr int R = RD::r(P - 1), Q = NN / R, WL = RD::W(P - 1);
        constexpr int NB = cdiv(KB * Q, kNT);
        // every multiplier load of the thread's butterflies first: one L2 latency per chunk, not one per butterfly.
        // Buffer loads: one VGPR offset per butterfly, the multiplier's row m W_L H as a constant SGPR offset
        // (global loads would hold a 64-bit address per multiplier: 2 R NB VGPRs next to the spectrum)
        const int t0 = tid();
        const rsrc_t rc = make_rsrc(Ct, (unsigned)(H * NN * 4));
        float cm[NB][R];
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int idx = t0 + u * kNT;
            if (u < NB - 1 || idx < KB * Q) {
                const int b = idx / KB, f = idx - b * KB;
                const unsigned vo = 4u * (unsigned)(dlast<NN>(b) * H + kc0 + (f < kc ? f : 0));
#pragma unroll
                for (int m = 0; m < R; ++m) cm[u][m] = bld1(rc, vo, 4u * (unsigned)(m * WL * H));
            }
        }
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int idx = t0 + u * kNT;
            if (u < NB - 1 || idx < KB * Q) {
                const int b = idx / KB, f = idx - b * KB;
                float2 v[R];
#pragma unroll
                for (int m = 0; m < R; ++m) v[m] = a.ld(f, b * R + m);
                dftR<R, false>(v);
#pragma unroll
                for (int m = 0; m < R; ++m) v[m] = cscale(v[m], cm[u][m]);
                dftR<R, true>(v);
#pragma unroll
                for (int m = 0; m < R; ++m) a.st(f, b * R + m, v[m]);
            }
        }
    }
    __syncthreads();
    dit_passes<NN, 0, P - 1, true, false, FS>(KB, th.twn, a);
}
template <int MM, int NN, int C, int NREG>
__device__ __forceinline__ void column_chunk(float2 (&S)[NREG], const Thr& th0, const float* __restrict__ Ct) {
    using G = Geo<MM, NN>;
    const Thr th = thr_of<MM, NN>(th0.buf, th0.twm, th0.twn);
    constexpr int kc0 = C * G::KBC, kc1 = imin(G::H, kc0 + G::KBC);
    column_stage<MM, NN, C>(S, th);
    column_passes<MM, NN>(kc0, kc1 - kc0, th, Ct);
    column_unstage<MM, NN, C>(S, th);
    __syncthreads();
}
// all column chunks of an iteration
template <int MM, int NN, int NREG>
__device__ __forceinline__ void column_phase(float2 (&S)[NREG], const Thr& th0, const float* __restrict__ Ct) {
    using G = Geo<MM, NN>;
    if constexpr (RS_COLSHARE && G::NCC > 1) {
        // chunk c is always register group 0: after each chunk the groups rotate by one (NCC rotations = identity),
        // so every register is written unconditionally (no phi of an old and a new value per register)
        constexpr int NR = G::NR;
#pragma unroll 1
        for (int c = 0; c < G::NCC; ++c) {
            const Thr th = thr_of<MM, NN>(th0.buf, th0.twm, th0.twn);
            const int kc0 = __builtin_amdgcn_readfirstlane(c) * G::KBC;
            const int kc = imin(G::H, kc0 + G::KBC) - kc0;
            column_stage<MM, NN, 0>(S, th, kc);
            column_passes<MM, NN>(kc0, kc, th, Ct);
            column_unstage<MM, NN, 0>(S, th, kc);
            __syncthreads();
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const float2 t0 = S[r];
#pragma unroll
                for (int g = 0; g + 1 < G::NCC; ++g) S[g * NR + r] = S[(g + 1) * NR + r];
                S[(G::NCC - 1) * NR + r] = t0;
            }
        }
    } else {
        static_for<0, G::NCC>([&](auto ic) { column_chunk<MM, NN, decltype(ic)::value>(S, th0, Ct); });
    }
}

// ---- line phase, chunk C: lines [jc0, jc1) ---------------------------------------------------------------
// Lines are held as complex pairs z_f = line 2f + i line 2f+1 (both spectra with their Hermitian
// extensions folded in, then both real lines after the inverse), M float2 per pair.  Update mode stages
// the chunk plus the halo pairs (jc0 - 2, jc0 - 1) and (jc1, jc1 + 1): pair u / 2 of staged line u.
// kIsoB / kIsoA: the isotropic solve's two halves of an iteration (resident_iso_kernel below)
enum Mode { kInit = 0, kUpdate = 1, kFinal = 2, kIsoB = 3, kIsoA = 4 };

struct LineArgs {
    const float* hty;     // this plane's H^T y
    const float* so;      // s_old (channel 0; channel 1 at + MN), unused when first
    float* sn;            // s_new
    float* xo;            // x out (final)
    float tau, rho;
    bool first;
    const float* fm;      // isotropic: the batch's BT factor map f_k (M x N, L2-resident)
    float* q;             // isotropic: this plane's q = s1^2 + s2^2 of s_{k+1} (the batch norm's input)
    float l0[4];          // update: s channel 0 of line 0 (wave 0's lanes), held from chunk 0 to the last chunk
};

__device__ __forceinline__ float2 lane_swap(float2 v) {   // value of lane t ^ 1 (DPP quad_perm [1, 0, 3, 2])
    const int x = __builtin_amdgcn_mov_dpp(__float_as_int(v.x), 0xB1, 0xF, 0xF, true);
    const int y = __builtin_amdgcn_mov_dpp(__float_as_int(v.y), 0xB1, 0xF, 0xF, true);
    return make_float2(__int_as_float(x), __int_as_float(y));
}

// Per-thread constants of the pair staging / separation (branch-free, so a register's store is one
// ds_write at a compile-time offset from the thread's base).  At DC and Nyquist both lanes of a pair write
// the same slot with the same value (the real parts of both lines).
struct ZLane {
    int slot;        // z slot this lane writes: k (even line) or M - k (odd line)
    float sgn;       // +1 even, -1 odd
    float im;        // 0 at DC / Nyquist (a real line's inverse keeps only the real parts), else 1
    bool odd;
};
template <int MM>
__device__ __forceinline__ ZLane zlane(int k, bool odd) {
    const bool edge = k == 0 || 2 * k == MM;
    return {odd ? (edge ? k : MM - k) : k, odd ? -1.0f : 1.0f, edge ? 0.0f : 1.0f, odd};
}
// own X_j(k) and the partner lane's X_{j^1}(k) -> z value: even line z[k] = X_2f + i X_2f+1,
// odd line z[M - k] = conj X_2f + i conj X_2f+1 (Hermitian extension)
__device__ __forceinline__ float2 zval(float2 x, float2 o, const ZLane& zl) {
    const float2 a = zl.odd ? o : x;   // X_2f
    const float2 b = zl.odd ? x : o;   // X_2f+1
    return make_float2(fmaf(-zl.sgn * zl.im, b.y, a.x), fmaf(zl.sgn * zl.im, a.y, b.x));
}
// separation from z (bin k) and z' = z(M - k): even line X = (z + conj z') / 2, odd X = (z - conj z') / (2i)
__device__ __forceinline__ float2 zsep(float2 z, float2 zm, bool odd) {
    const float px = odd ? z.y : z.x, py = odd ? -z.x : z.y;
    const float qx = odd ? zm.y : zm.x, qy = odd ? zm.x : -zm.y;
    return make_float2(0.5f * (px + qx), 0.5f * (py + qy));
}

// hs[C NCC + c]: for C >= 1 chunk C's halo-A register (lines jc0 - 2, jc0 - 1) of column chunk c, for C = 0 the
// register of lines 0, 1 (the last chunk's halo B), saved before the update phase: by the time a chunk stages
// them, the chunk that owns those lines has already replaced them with the next iteration's spectra.
template <int MM, int NN, int C, int MODE, int NREG, int NH>
__device__ __forceinline__ void line_chunk(float2 (&S)[NREG], const float2 (&hs)[NH], const Thr& th0, LineArgs& a) {
    using G = Geo<MM, NN>;
    const Thr th = thr_of<MM, NN>(th0.buf, th0.twm, th0.twn);
    using RD = Rad<MM>;
    constexpr int LS = G::LS, P = RD::P, NR = G::NR, NCC = G::NCC, KBC = G::KBC, H = G::H;
    constexpr int jc0 = C * G::TL, jc1 = imin(NN, jc0 + G::TL), T = jc1 - jc0;
    constexpr int rc0 = jc0 / LS, rc1 = cdiv(jc1, LS);   // the chunk's registers (the last may hold lines >= NN)
    constexpr int HP = (MODE == kUpdate || MODE == kIsoA) ? 1 : 0;   // halo pairs either side
    constexpr int NP = T / 2 + 2 * HP;            // pairs staged
    float2* buf = th.buf;
    float* Xf = reinterpret_cast<float*>(buf);
    const Acc<MM> al{buf};
    const bool odd = th.jt & 1;

    if constexpr (MODE != kInit && MODE != kIsoB) {
        // ---- S -> z pairs (stores only), inverse DIF (x at dpos order) ----
        float2* zb0 = buf + (th.jt >> 1) * MM;   // + z slot + pair offset of register r
        static_for<0, NCC>([&](auto ic) {
            constexpr int c = decltype(ic)::value;
            const int k = c * KBC + th.kk;
            const bool kv = th.act && k < H;      // lanes past the last chunk's bins store nothing
            const ZLane zl = zlane<MM>(k, odd);
            float2* zb = zb0 + zl.slot;
#pragma unroll
            for (int r = rc0; r < rc1; ++r) {
                const float2 z = zval(S[c * NR + r], lane_swap(S[c * NR + r]), zl);
                if (kv && (r < rc1 - 1 || r * LS + th.jt < jc1)) zb[((r * LS - jc0) / 2 + HP) * MM] = z;
            }
            if constexpr (HP) {
                constexpr int hA = (jc0 + NN - 2) % NN, hB = jc1 % NN;   // even lines: pairs (hA, hA+1), (hB, hB+1)
                const float2 sA = C >= 1 ? hs[C * NCC + c] : S[c * NR + hA / LS];
                const float2 zA = zval(sA, lane_swap(sA), zl);
                if (kv && (th.jt >> 1) == (hA % LS) / 2) buf[zl.slot] = zA;
                const float2 sB = (C == G::NLC - 1 && G::NLC > 1) ? hs[c] : S[c * NR + hB / LS];
                const float2 zB = zval(sB, lane_swap(sB), zl);
                if (kv && (th.jt >> 1) == (hB % LS) / 2) buf[(NP - 1) * MM + zl.slot] = zB;
            }
        });
        __syncthreads();
        dif_passes<MM, 0, P, true, true, MM>(NP, th.twm, al);
    }

    if constexpr (MODE == kFinal) {
        // x rows out in natural pixel order (pair (j - jc0) / 2, real part for even j)
        float* xo = a.xo + (size_t)jc0 * MM;
        for (int idx = tid(); idx < T * MM; idx += kNT) {
            const int u = idx / MM, i = idx - u * MM;
            xo[idx] = Xf[2 * ((u >> 1) * MM + dpos<MM>(i)) + (u & 1)];
        }
        __syncthreads();
        return;
    }

    if constexpr (MODE == kIsoA) {
        // ---- isotropic A phase: s_{k+1} = D x_{k+1} + u_k, u_k = s_k - f_k s_k (z = f s, ops.jl:10; first: u = 0),
        // stored, and q = s1^2 + s2^2 of the pixel for the batch norm.  x of line j - 1 (channel 0, dim 2) and pixel
        // i - 1 (channel 1, dim 1) from the staged rows (the halo pair holds lines jc0 - 2, jc0 - 1).  No forward
        // transform: the next launch's B phase forms the spectrum from s_{k+1}.  Rows walked per wave as in the
        // anisotropic update (GP pixels per lane, buffer loads RS_PDI rows ahead in a ring that never moves); the
        // first launch reads s_k and f_k through zero-size resources (every load 0: u = 0, bitwise the old branch).
        // In place (s_in = s_out) is safe: a row is read RS_PDI rows before its own wave rewrites it.
        constexpr int GP = G::GP, QG = G::QG;
        constexpr unsigned MN = (unsigned)MM * NN;
        using PV = Vg<GP>;
        const RowLanes<MM> rl;
        const int w = __builtin_amdgcn_readfirstlane(tid() >> 6);
        const int ua = 2 + (w * T) / 8, ub = 1 + ((w + 1) * T) / 8;
        const unsigned live = a.first ? 0u : MN * 4;
        const rsrc_t rso = make_rsrc(a.so, 2 * live), rfm = make_rsrc(a.fm, live), rsn = make_rsrc(a.sn, 2 * MN * 4),
                     rq = make_rsrc(a.q, MN * 4);
        auto row = [&](int u) { return 2 * (u >> 1) * MM + (u & 1); };
        struct AIn {
            PV f, o0, o1;
        };
        const rsrc_t rnone = make_rsrc(a.sn, 0u);   // rows past the wave's last: not loaded (as in the update)
        auto aload = [&](AIn (&g)[QG], int u) {
            const unsigned oj = 4u * (unsigned)((jc0 + u - 2) * MM);
            const rsrc_t rf = u <= ub ? rfm : rnone, rs = u <= ub ? rso : rnone;
#pragma unroll
            for (int q = 0; q < QG; ++q) {
                g[q].f = rl.template ld<GP>(rf, q, oj);
                g[q].o0 = rl.template ld<GP>(rs, q, oj);
                g[q].o1 = rl.template ld<GP>(rs, q, oj + 4 * MN);
            }
        };
        auto astep = [&](int u, const AIn (&cur)[QG]) {
            const unsigned oj = 4u * (unsigned)((jc0 + u - 2) * MM);
            const int ru = row(u), rp = row(u - 1);
#pragma unroll
            for (int q = 0; q < QG; ++q) {
                const PV xc = rl.template xget<GP>(Xf, ru, q), xp = rl.template xget<GP>(Xf, rp, q);
                const float xl = Xf[ru + rl.plo[q]];
                PV s0, s1, qq;
#pragma unroll
                for (int g = 0; g < GP; ++g) {
                    const float f = cur[q].f.v[g], o0 = cur[q].o0.v[g], o1 = cur[q].o1.v[g];
                    s0.v[g] = (xc.v[g] - xp.v[g]) + (o0 - f * o0);
                    s1.v[g] = (xc.v[g] - (g == 0 ? xl : xc.v[g > 0 ? g - 1 : 0])) + (o1 - f * o1);
                    qq.v[g] = s0.v[g] * s0.v[g] + s1.v[g] * s1.v[g];
                }
                rl.template st<GP>(rsn, q, oj, s0);
                rl.template st<GP>(rsn, q, oj + 4 * MN, s1);
                rl.template st<GP>(rq, q, oj, qq);
            }
        };
        if (ub >= ua) {
            constexpr int NS = RS_PDI + 1;
            AIn pf[NS][QG];
#pragma unroll
            for (int d = 0; d < RS_PDI; ++d) aload(pf[d], ua + d);
#pragma unroll 1
            for (int u0 = ua; u0 <= ub; u0 += NS) {
                static_for<0, NS>([&](auto id) {
                    constexpr int d = decltype(id)::value;
                    const int u = u0 + d;
                    if (u <= ub) {
                        aload(pf[(d + RS_PDI) % NS], u + RS_PDI);
                        astep(u, pf[d]);
                    }
                });
            }
        }
        __syncthreads();
        return;
    }

    if constexpr (MODE == kUpdate) {
        // ---- row update: wave w walks staged lines ua .. ub (staged line u = line jc0 + u - 2) ----
        // A lane takes GP neighbouring pixels i0 = GP (lane + 64 q) .. i0 + GP - 1 (GP = 2 for lines longer than
        // 64: 8-byte buffer loads and stores, so a row costs 3 loads + 2 stores per slice of 128 pixels).  gfx950
        // counts loads and stores in one 6-bit vmcnt, so at most 63 of them are in flight per wave: with 4-byte
        // accesses that held about 3 rows ahead and the update ran at the HBM latency per 3 rows (pairs: 250^2
        // 2.68 -> 2.62 ms, 240^2 3.11 -> 2.43, 192^2 1.73 -> 1.42, 128^2 0.78 -> 0.70; at 64 and 32 points a
        // pair per lane leaves half the lanes idle: 0.59 -> 0.66 and 0.50 -> 0.64, so those keep GP = 1).
        // Global traffic through buffer resources: the row offset is wave-uniform (soffset), the lane's pixel
        // offset a per-lane constant (voffset).
        constexpr int GP = G::GP, QG = G::QG;
        constexpr unsigned MN = (unsigned)MM * NN;
        using PV = Vg<GP>;
        const int t = tid();
        const int w = __builtin_amdgcn_readfirstlane(t >> 6);
        const int lane = t & 63;
        const int ua = 2 + (w * T) / 8, ub = 1 + ((w + 1) * T) / 8;
        const float tau = a.tau, rho = a.rho;
        const rsrc_t rso = make_rsrc(a.so, a.first ? 0u : 2 * MN * 4), rsn = make_rsrc(a.sn, 2 * MN * 4),
                     rh = make_rsrc(a.hty, MN * 4), rnone = make_rsrc(a.sn, 0u);
        // LDS float offsets (x at dpos order within a pair row) of the lane's pixels and of the first one's left
        // neighbour (the others' left neighbours are the lane's own pixels)
        int po[QG][GP], plo[QG];
#pragma unroll
        for (int q = 0; q < QG; ++q) {
            const int i0 = GP * (lane + 64 * q) < MM ? GP * (lane + 64 * q) : 0;
#pragma unroll
            for (int g = 0; g < GP; ++g) po[q][g] = 2 * dpos<MM>(i0 + g);
            plo[q] = 2 * dpos<MM>(i0 == 0 ? MM - 1 : i0 - 1);
        }
        constexpr unsigned SL = 256 * GP;                    // bytes per slice: the instruction's immediate offset
        const unsigned gl = 4u * GP * (unsigned)lane;
        auto row = [&](int u) { return 2 * (u >> 1) * MM + (u & 1); };
        auto valid = [&](int q) { return q < QG - 1 || GP * (lane + 64 * q) < MM; };
        // HBM stores of lanes past the row's end go to a lane offset beyond the buffer (dropped by the buffer
        // unit): no exec-mask branch around them
        const unsigned glst = GP * (lane + 64 * (QG - 1)) < MM ? gl : 0x80000000u;
        auto gst = [&](int q) { return q < QG - 1 ? gl : glst; };
        auto ld = [&](rsrc_t r, int q, unsigned so) { return PV::load(r, gl + SL * q, so); };
        auto st = [&](rsrc_t r, int q, unsigned so, const PV& v) { v.store(r, gst(q) + SL * q, so); };
        auto xget = [&](int rbase, int q) {
            PV x;
#pragma unroll
            for (int g = 0; g < GP; ++g) x.v[g] = Xf[rbase + po[q][g]];
            return x;
        };
        auto put = [&](int q, int rbase, const PV& v) {
            if (valid(q)) {
#pragma unroll
                for (int g = 0; g < GP; ++g) Xf[rbase + po[q][g]] = v.v[g];
            }
        };
        // the wave's scratch rows (float offsets from Xf): first row at + 0, last row at + 1, stride 2 like a pair
        constexpr bool SC = G::kScr;
        const int scr = 2 * G::BUF + w * 2 * MM;
        PV vf[QG], vl[QG];
        PV s0a[QG];   // RS_INPLACE: s channel 0 of the wave's first row, stored after the barrier
        if (ub >= ua) {
            PV w0c[QG];
            {
                const int j = jc0 + ua - 2;
                const int ru = row(ua), rm = row(ua - 1);
                const unsigned so = 4u * (unsigned)(j * MM);
#pragma unroll
                for (int q = 0; q < QG; ++q) {
                    const PV o = ld(rso, q, so), xa = xget(ru, q), xb = xget(rm, q);
                    PV s0;
#pragma unroll
                    for (int g = 0; g < GP; ++g) s0.v[g] = (xa.v[g] - xb.v[g]) + clipf(o.v[g], tau);
#if RS_INPLACE
                    // stored after the block barrier below: the previous wave still reads this row's old channel 0
                    // (its last row's s0 of line j + 1), and in place that would be the new value
                    s0a[q] = s0;
#else
                    st(rsn, q, so, s0);
#endif
#pragma unroll
                    for (int g = 0; g < GP; ++g) w0c[q].v[g] = prox_w(s0.v[g], tau);
                }
            }
            struct GIn {
                PV a0n, a1, h;
            };
            // (the first iteration reads s_old through a zero-size resource: every load returns 0, no branch)
            // rows past the wave's last are not loaded at all (a zero-size resource, a scalar select): the ring's
            // look-ahead would otherwise read the next wave's rows (L2 hits) and, at a chunk's end, the next
            // chunk's (HBM again, long evicted when that chunk runs)
            const rsrc_t rnh = make_rsrc(a.hty, 0u);
            auto gload = [&](GIn (&gi)[QG], int u) {
                const int j = jc0 + u - 2;
                const int jn = j + 1 == NN ? 0 : j + 1;
                const unsigned oj = 4u * (unsigned)(j * MM), on = 4u * (unsigned)(jn * MM);
                const bool in = u <= ub;
                const rsrc_t rhu = in ? rh : rnh, rsu = in ? rso : rnone;
#pragma unroll
                for (int q = 0; q < QG; ++q) {
                    gi[q].h = ld(rhu, q, oj);
                    gi[q].a0n = ld(rsu, q, on);
                    gi[q].a1 = ld(rsu, q, oj + 4 * MN);
                }
            };
            auto step = [&](int u, const GIn (&cur)[QG]) {
                const int j = jc0 + u - 2;
                const int jn = j + 1 == NN ? 0 : j + 1;
                const unsigned oj = 4u * (unsigned)(j * MM), on = 4u * (unsigned)(jn * MM);
                const int ru = row(u), rn = row(u + 1);
                // every read of the row before any v is written over it: lanes read their neighbours' pixels
                PV xc[QG], xn[QG];
                float xl[QG];
#pragma unroll
                for (int q = 0; q < QG; ++q) {
                    xc[q] = xget(ru, q);
                    xn[q] = xget(rn, q);
                    xl[q] = Xf[ru + plo[q]];
                }
                PV w0n[QG], w1[QG];
#pragma unroll
                for (int q = 0; q < QG; ++q) {
                    PV s0n, s1;
#pragma unroll
                    for (int g = 0; g < GP; ++g) {
                        s0n.v[g] = (xn[q].v[g] - xc[q].v[g]) + clipf(cur[q].a0n.v[g], tau);
                        s1.v[g] = (xc[q].v[g] - (g == 0 ? xl[q] : xc[q].v[g > 0 ? g - 1 : 0])) + clipf(cur[q].a1.v[g], tau);
                    }
                    // s0 of line j + 1: the next wave's (or chunk's) first row, which it stores itself -- not
                    // from the last row (a zero-size resource drops the store)
                    st(u < ub ? rsn : rnone, q, on, s0n);
                    st(rsn, q, oj + 4 * MN, s1);
#pragma unroll
                    for (int g = 0; g < GP; ++g) {
                        w0n[q].v[g] = prox_w(s0n.v[g], tau);
                        w1[q].v[g] = prox_w(s1.v[g], tau);
                    }
                }
                // w of channel 1 at the pixel right of each: the lane's own next pixel, and for its last pixel the
                // next lane's first (lane 63: lane 0 of the next slice; the row's last pixel wraps to pixel 0) --
                // the value the neighbour computed, not a second evaluation of it
                float sh[QG];
#pragma unroll
                for (int q = 0; q < QG; ++q)
                    sh[q] = __int_as_float(__builtin_amdgcn_ds_bpermute(4 * ((lane + 1) & 63), __float_as_int(w1[q].v[0])));
                const float p0 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(w1[0].v[0])));
#pragma unroll
                for (int q = 0; q < QG; ++q) {
                    const float nx = q + 1 < QG ? sh[q + 1 < QG ? q + 1 : q] : p0;
                    const float wlast = GP * (lane + 64 * q) + GP == MM ? p0 : (lane == 63 ? nx : sh[q]);
                    PV v;
#pragma unroll
                    for (int g = 0; g < GP; ++g) {
                        const float w1r = g + 1 < GP ? w1[q].v[g + 1 < GP ? g + 1 : g] : wlast;
                        v.v[g] = fmaf(rho, (w0c[q].v[g] - w0n[q].v[g]) + (w1[q].v[g] - w1r), cur[q].h.v[g]);
                    }
                    w0c[q] = w0n[q];
                    if constexpr (SC) {
                        put(q, u == ua ? scr : u == ub ? scr + 1 : ru, v);   // uniform: a scalar select
                    } else {
                        if (u == ua) vf[q] = v;
                        else if (u == ub) vl[q] = v;
                        else put(q, ru, v);
                    }
                }
            };
            // rows u + 1 .. u + RS_PD in flight while row u is computed (loads past the chunk read rows the
            // next chunk or another wave owns, or beyond the plane, where the buffer returns 0: never used).
            // RS_PD + 1 ring slots, the loop unrolled by that many rows: row ua + i lives in slot i % NS, a
            // compile-time index in every unrolled step, so the ring never moves a register (rotating it
            // cost 77 v_mov per row, a third of the row's VALU)
            constexpr int NS = RS_PD + 1;
            GIn pf[NS][QG];
#pragma unroll
            for (int d = 0; d < RS_PD; ++d) gload(pf[d], ua + d);
#pragma unroll 1
            for (int u0 = ua; u0 <= ub; u0 += NS) {
                static_for<0, NS>([&](auto id) {
                    constexpr int d = decltype(id)::value;
                    const int u = u0 + d;
                    if (u <= ub) {
                        gload(pf[(d + RS_PD) % NS], u + RS_PD);
                        step(u, pf[d]);
                    }
                });
            }
        }
        __syncthreads();
        if (ub >= ua) {
#pragma unroll
            for (int q = 0; q < QG; ++q) {
                put(q, row(ua), SC ? xget(scr, q) : vf[q]);
                if (ub > ua) put(q, row(ub), SC ? xget(scr + 1, q) : vl[q]);
            }
        }
#if RS_INPLACE
        // the first rows' channel 0 (every wave's row loop, which reads the next wave's first row, is done).  Line 0
        // (chunk 0, wave 0) waits for the last chunk when there are several: that chunk's last wave reads line 0's
        // old channel 0 as its line j + 1
        {
            static_assert(QG * GP <= 4, "LineArgs::l0 holds 4 floats");
            const unsigned sof = 4u * (unsigned)((jc0 + ua - 2) * MM);
            if constexpr (C == 0 && G::NLC > 1) {
                if (w == 0) {
#pragma unroll
                    for (int q = 0; q < QG; ++q)
#pragma unroll
                        for (int g = 0; g < GP; ++g) a.l0[q * GP + g] = s0a[q].v[g];
                } else if (ub >= ua) {
#pragma unroll
                    for (int q = 0; q < QG; ++q) st(rsn, q, sof, s0a[q]);
                }
            } else {
                if (ub >= ua) {
#pragma unroll
                    for (int q = 0; q < QG; ++q) st(rsn, q, sof, s0a[q]);
                }
            }
            if constexpr (C == G::NLC - 1 && G::NLC > 1) {
                if (w == 0) {
#pragma unroll
                    for (int q = 0; q < QG; ++q) {
                        PV l;
#pragma unroll
                        for (int g = 0; g < GP; ++g) l.v[g] = a.l0[q * GP + g];
                        st(rsn, q, 0u, l);
                    }
                }
            }
        }
#endif
        __syncthreads();
        // ---- forward DIT of the chunk's pairs (v at dpos order -> natural z) ----
        dit_passes<MM, 0, P, false, true, MM>(T / 2, th.twm, Acc<MM>{buf + MM});
    } else if constexpr (MODE == kIsoB) {
        // isotropic B phase: v = H^T y + rho D^T w, w = z - u = f s - (s - f s) of s_k and f_k (ops.jl:10, 168), into
        // the pairs at dpos order (element of line jc0 + u, pixel i at float 2 ((u / 2) M + dpos(i)) + u % 2).
        // D^T needs w of line j + 1 (channel 0) and of pixel i + 1 (channel 1): a wave walks its rows carrying f and
        // channel 0's w of the row below into the next step, and takes channel 1's w of pixel i + 1 from the lane
        // that computed it -- each w evaluated once, bitwise the values of a per-element evaluation.
        constexpr int GP = G::GP, QG = G::QG;
        constexpr unsigned MN = (unsigned)MM * NN;
        using PV = Vg<GP>;
        const RowLanes<MM> rl;
        const int lane = tid() & 63;
        const int w = __builtin_amdgcn_readfirstlane(tid() >> 6);
        const int ua = (w * T) / 8, ub = ((w + 1) * T) / 8 - 1;
        const rsrc_t rso = make_rsrc(a.so, 2 * MN * 4), rfm = make_rsrc(a.fm, MN * 4), rh = make_rsrc(a.hty, MN * 4);
        auto row = [&](int u) { return 2 * (u >> 1) * MM + (u & 1); };
        auto wof = [](float f, float sv) { return f * sv - (sv - f * sv); };
        auto off = [&](int u) {   // byte offset of line jc0 + u (periodic)
            const int j = jc0 + u;
            return 4u * (unsigned)((j >= NN ? j - NN : j) * MM);
        };
        struct BIn {
            PV fn, s0n, s1, h;   // f and s channel 0 of line j + 1; s channel 1 and H^T y of line j
        };
        const rsrc_t rnone = make_rsrc(a.hty, 0u);   // rows past the wave's last: not loaded (as in the update)
        auto bload = [&](BIn (&g)[QG], int u) {
            const unsigned oj = off(u), on = off(u + 1);
            const bool in = u <= ub;
            const rsrc_t rf = in ? rfm : rnone, rs = in ? rso : rnone, rhh = in ? rh : rnone;
#pragma unroll
            for (int q = 0; q < QG; ++q) {
                g[q].fn = rl.template ld<GP>(rf, q, on);
                g[q].s0n = rl.template ld<GP>(rs, q, on);
                g[q].s1 = rl.template ld<GP>(rs, q, oj + 4 * MN);
                g[q].h = rl.template ld<GP>(rhh, q, oj);
            }
        };
        PV fc[QG], w0c[QG];   // f and channel 0's w of the current line
        auto bstep = [&](int u, const BIn (&cur)[QG]) {
            PV w1[QG];
#pragma unroll
            for (int q = 0; q < QG; ++q)
#pragma unroll
                for (int g = 0; g < GP; ++g) w1[q].v[g] = wof(fc[q].v[g], cur[q].s1.v[g]);
            float sh[QG];
#pragma unroll
            for (int q = 0; q < QG; ++q)
                sh[q] = __int_as_float(__builtin_amdgcn_ds_bpermute(4 * ((lane + 1) & 63), __float_as_int(w1[q].v[0])));
            const float p0 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(w1[0].v[0])));
#pragma unroll
            for (int q = 0; q < QG; ++q) {
                const float nx = q + 1 < QG ? sh[q + 1 < QG ? q + 1 : q] : p0;
                const float wlast = GP * (lane + 64 * q) + GP == MM ? p0 : (lane == 63 ? nx : sh[q]);
                PV v;
#pragma unroll
                for (int g = 0; g < GP; ++g) {
                    const float w0n = wof(cur[q].fn.v[g], cur[q].s0n.v[g]);
                    const float w1r = g + 1 < GP ? w1[q].v[g + 1 < GP ? g + 1 : g] : wlast;
                    v.v[g] = fmaf(a.rho, (w0c[q].v[g] - w0n) + (w1[q].v[g] - w1r), cur[q].h.v[g]);
                    w0c[q].v[g] = w0n;
                }
                fc[q] = cur[q].fn;
                rl.put(Xf, q, row(u), v);
            }
        };
        if (ub >= ua) {
            {
                const unsigned oj = off(ua);
#pragma unroll
                for (int q = 0; q < QG; ++q) {
                    fc[q] = rl.template ld<GP>(rfm, q, oj);
                    const PV s0 = rl.template ld<GP>(rso, q, oj);
#pragma unroll
                    for (int g = 0; g < GP; ++g) w0c[q].v[g] = wof(fc[q].v[g], s0.v[g]);
                }
            }
            constexpr int NS = RS_PDI + 1;
            BIn pf[NS][QG];
#pragma unroll
            for (int d = 0; d < RS_PDI; ++d) bload(pf[d], ua + d);
#pragma unroll 1
            for (int u0 = ua; u0 <= ub; u0 += NS) {
                static_for<0, NS>([&](auto id) {
                    constexpr int d = decltype(id)::value;
                    const int u = u0 + d;
                    if (u <= ub) {
                        bload(pf[(d + RS_PDI) % NS], u + RS_PDI);
                        bstep(u, pf[d]);
                    }
                });
            }
        }
        __syncthreads();
        dit_passes<MM, 0, P, false, true, MM>(T / 2, th.twm, al);
    } else {
        // kInit: the first iteration's v = H^T y, from HBM into the pairs at dpos order
        for (int idx = tid(); idx < T * MM / 2; idx += kNT) {
            const int f = idx / MM, i = idx - f * MM;
            const float* hp = a.hty + (size_t)(jc0 + 2 * f) * MM + i;
            buf[f * MM + dpos<MM>(i)] = make_float2(hp[0], hp[MM]);
        }
        __syncthreads();
        dit_passes<MM, 0, P, false, true, MM>(T / 2, th.twm, al);
    }
    // ---- half spectra separated into S: X_2f = (z + conj z(-k)) / 2, X_2f+1 = (z - conj z(-k)) / (2i) ----
    // Every thread, every register of the chunk: lanes past the last column chunk's bins take bin H - 1 and
    // padding lines (j >= NN) read pairs inside the buffer; neither value is ever used.
    {
        const float2* Zb = buf + ((th.jt >> 1) + HP) * MM;   // + pair offset of register r
        static_for<0, NCC>([&](auto ic) {
            constexpr int c = decltype(ic)::value;
            const int k = imin(c * KBC + th.kk, H - 1), km = k == 0 ? 0 : MM - k;
#pragma unroll
            for (int r = rc0; r < rc1; ++r) {
                const float2* Z = Zb + ((r * LS - jc0) / 2) * MM;
                S[c * NR + r] = zsep(Z[k], Z[km], odd);
#if RS_PINSEP
                // formed here: left free, the compiler sinks zsep to the next use (the next iteration) and keeps
                // both loaded halves live instead, twice the registers
                __asm__ volatile("" : "+v"(S[c * NR + r].x), "+v"(S[c * NR + r].y));
#endif
            }
        });
    }
    __syncthreads();
}

// ---- the kernel: one workgroup per plane, all K iterations ---------------------------------------------------
template <int MM, int NN>
__global__ __launch_bounds__(kNT) void resident_kernel(const float* __restrict__ hty_all, float* __restrict__ sA,
                                                       float* __restrict__ sB, float* __restrict__ traj, size_t traj_stride,
                                                       float* __restrict__ x_all, const float* __restrict__ Ct,
                                                       const float2* __restrict__ twM, const float2* __restrict__ twN,
                                                       const float* __restrict__ prm, int maxit) {
    using G = Geo<MM, NN>;
    constexpr int NREG = G::NREG, NR = G::NR, NCC = G::NCC;
    constexpr size_t MN = (size_t)MM * NN;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float2* twm = reinterpret_cast<float2*>(smem_raw);
    float2* twn = twm + MM;
    fill_twiddles<MM>(twm, twM, kNT);
    fill_twiddles<NN>(twn, twN, kNT);
    const size_t plane = blockIdx.x;
    const unsigned t = threadIdx.x;
    Thr th;
    th.buf = twn + NN;
    th.twm = twm;
    th.twn = twn;
    th.kk = (int)(t / G::LS);
    th.jt = (int)(t % G::LS);
    th.act = t < (unsigned)(G::KBC * G::LS);
    LineArgs la;
    la.hty = hty_all + plane * MN;
    la.xo = x_all + plane * MN;
    la.tau = prm[0];
    la.rho = prm[1];
    la.so = nullptr;
    la.sn = nullptr;
    la.first = true;
    la.fm = nullptr;   // isotropic modes only
    la.q = nullptr;
    float2 S[NREG];
#pragma unroll
    for (int r = 0; r < NREG; ++r) S[r] = make_float2(0.f, 0.f);
    __syncthreads();
    float2 hs[G::NLC * NCC];
    static_for<0, G::NLC>([&](auto ic) { line_chunk<MM, NN, decltype(ic)::value, kInit>(S, hs, th, la); });
#pragma unroll 1
    for (int it = 1; it <= maxit; ++it) {
        column_phase<MM, NN>(S, th, Ct);
        if (it == maxit) {
            static_for<0, G::NLC>([&](auto ic) { line_chunk<MM, NN, decltype(ic)::value, kFinal>(S, hs, th, la); });
            break;
        }
        float* sn;
        const float* so;
        if (traj) {
            sn = traj + (size_t)(it - 1) * traj_stride;
            so = it >= 2 ? traj + (size_t)(it - 2) * traj_stride : sn;
        } else {
            sn = (!RS_INPLACE && (it & 1)) ? sA : sB;
            so = RS_INPLACE ? sn : (it & 1) ? sB : sA;
        }
        la.sn = sn + plane * 2 * MN;
        la.so = so + plane * 2 * MN;
        la.first = it == 1;
#pragma unroll
        for (int c = 0; c < NCC; ++c) hs[c] = S[c * NR];
        static_for<1, G::NLC>([&](auto ic) {
            constexpr int C = decltype(ic)::value;
#pragma unroll
            for (int c = 0; c < NCC; ++c) hs[C * NCC + c] = S[c * NR + (C * G::TL - 2) / G::LS];
        });
        static_for<0, G::NLC>([&](auto ic) { line_chunk<MM, NN, decltype(ic)::value, kUpdate>(S, hs, th, la); });
    }
}

// ---- the isotropic solve: one launch per iteration ------------------------------------------------------------
// BT couples every plane through the per-pixel batch norm (ops.jl:6,10), so an iteration cannot finish inside one
// workgroup.  As plane256_iso_kernel does at 256^2 (plane_iso.hip), each iteration k = 0 .. K-1 is one launch,
// split at the norm:  B phase (k > 0; k = 0 starts from v = H^T y): v from s_k and f_k, line forward;
// column phase (x C, ops.jl:86); line inverse -> x_{k+1}; A phase: s_{k+1} = D x_{k+1} + (s_k - f_k s_k) stored,
// q per pixel (k = K - 1 writes x instead).  Between launches the 2-pass path's norm kernel (iso_r over the
// planes' q, or the sharded sum / reducer / factor) forms f_{k+1}.  The spectrum never leaves the CU within a
// launch; per pixel and iteration HBM moves s_k twice (B, A) and s_{k+1} once, H^T y and q: 32 B against the
// 2-pass step's 44 and four launches.
template <int MM, int NN>
__global__ __launch_bounds__(kNT) void resident_iso_kernel(const float* __restrict__ hty_all, const float* s_in,
                                                           float* s_out, const float* __restrict__ fmap,
                                                           float* __restrict__ q_all, float* __restrict__ x_all,
                                                           const float* __restrict__ Ct, const float2* __restrict__ twM,
                                                           const float2* __restrict__ twN, const float* __restrict__ prm,
                                                           int k, int K) {
    // s_in may equal s_out (in place, no trajectory): neither is __restrict__
    using G = Geo<MM, NN>;
    constexpr int NREG = G::NREG, NR = G::NR, NCC = G::NCC;
    constexpr size_t MN = (size_t)MM * NN;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float2* twm = reinterpret_cast<float2*>(smem_raw);
    float2* twn = twm + MM;
    fill_twiddles<MM>(twm, twM, kNT);
    fill_twiddles<NN>(twn, twN, kNT);
    const size_t plane = blockIdx.x;
    const unsigned t = threadIdx.x;
    Thr th;
    th.buf = twn + NN;
    th.twm = twm;
    th.twn = twn;
    th.kk = (int)(t / G::LS);
    th.jt = (int)(t % G::LS);
    th.act = t < (unsigned)(G::KBC * G::LS);
    LineArgs la;
    la.hty = hty_all + plane * MN;
    la.xo = x_all + plane * MN;
    la.tau = prm[0];
    la.rho = prm[1];
    la.so = s_in + plane * 2 * MN;
    la.sn = s_out + plane * 2 * MN;
    la.first = k == 0;
    la.fm = fmap;
    la.q = q_all + plane * MN;
    float2 S[NREG];
#pragma unroll
    for (int r = 0; r < NREG; ++r) S[r] = make_float2(0.f, 0.f);
    __syncthreads();
    float2 hs[G::NLC * NCC];
    if (k == 0) {
        static_for<0, G::NLC>([&](auto ic) { line_chunk<MM, NN, decltype(ic)::value, kInit>(S, hs, th, la); });
    } else {
        static_for<0, G::NLC>([&](auto ic) { line_chunk<MM, NN, decltype(ic)::value, kIsoB>(S, hs, th, la); });
    }
    column_phase<MM, NN>(S, th, Ct);
    if (k == K - 1) {
        static_for<0, G::NLC>([&](auto ic) { line_chunk<MM, NN, decltype(ic)::value, kFinal>(S, hs, th, la); });
        return;
    }
    // the A phase stages every chunk from S as it stands (no chunk's registers are rewritten in between), so the
    // halo registers are S itself
#pragma unroll
    for (int c = 0; c < NCC; ++c) hs[c] = S[c * NR];
    static_for<1, G::NLC>([&](auto ic) {
        constexpr int C = decltype(ic)::value;
#pragma unroll
        for (int c = 0; c < NCC; ++c) hs[C * NCC + c] = S[c * NR + (C * G::TL - 2) / G::LS];
    });
    static_for<0, G::NLC>([&](auto ic) { line_chunk<MM, NN, decltype(ic)::value, kIsoA>(S, hs, th, la); });
}

// ---- host side -----------------------------------------------------------------------------------------------
// Shapes compiled here (M = line length, N = lines): square smooth sides the 2-pass path serves, and the small
// power-of-two squares (the reference's 32 x 32 demo crops, src/ADMM_Deconv.jl:17-23; 64, 128)
#ifndef RS_SHAPES_OVERRIDE
#define RS_SHAPES(X) \
    X(250, 250) X(240, 240) X(200, 200) X(192, 192) X(160, 160) X(128, 128) X(120, 120) X(96, 96) X(64, 64) X(32, 32)
#else
#define RS_SHAPES(X) RS_SHAPES_OVERRIDE(X)
#endif

// Compiled shapes where the 2-pass kernels measured faster (ADMM_OPT_RESIDENT = 1 leaves them to the 2-pass
// path; 2 forces the resident kernel on every compiled shape).  None: no smooth shape since the spills went
// (round 4: 240^2 resident 77.8k img/s vs 74.2k 2-pass, profiles/r04_resident_shapes.jsonl), and the power-of-two
// squares beat their tuned 2-pass kernels too (128^2 x 256 0.91 vs 0.94 ms, 64^2 x 1024 0.68 vs 0.94, 32^2 x 2048
// 0.61 vs 1.59; profiles/r04_resident_pow2.jsonl).  Small batches are left to the 2-pass kernels by plan_paths.
#define RS_SLOWER(X)

// isotropic solve (resident_iso_kernel): shapes where the 2-pass isotropic kernels measured faster at a full wave of
// planes (profiles/r04_resident_iso_rows.jsonl, 256 planes, A / B phases as row walkers: 250^2 3.94 vs 5.78 ms,
// 200^2 2.70 vs 3.36, 160^2 1.78 vs 2.29, 120^2 1.04 vs 1.53, 96^2 0.81 vs 1.18, 64^2 x 512 0.80 vs 0.96, 32^2 x 512
// 0.60 vs 0.69; but 128^2 1.27 vs 1.20 against the tuned power-of-two kernels).  Below a wave the 2-pass kernels
// win (one launch per iteration with one plane per CU), which plan_paths' plane-count rule leaves to them.
#define RS_ISO_SLOWER(X) X(128, 128)

bool has_iso_shape(int M, int N, bool all) {
#define X(m, n) \
    if (!all && M == m && N == n) return false;
    RS_ISO_SLOWER(X)
#undef X
#define X(m, n) \
    if (M == m && N == n) return true;
    RS_SHAPES(X)
#undef X
    return false;
}

bool has_shape(int M, int N, bool all) {
#define X(m, n) \
    if (!all && M == m && N == n) return false;
    RS_SLOWER(X)
#undef X
#define X(m, n) \
    if (M == m && N == n) return true;
    RS_SHAPES(X)
#undef X
    return false;
}

int launch_iso(int M, int N, size_t planes, hipStream_t s, const float* hty, const float* s_in, float* s_out,
               const float* fmap, float* q, float* x_out, const float* Ct, const float2* twM, const float2* twN,
               const float* prm, int k, int K) {
#define X(m, n)                                                                                                  \
    if (M == m && N == n) {                                                                                      \
        constexpr size_t lds = Geo<m, n>::lds_bytes();                                                           \
        (void)hipFuncSetAttribute((const void*)resident_iso_kernel<m, n>,                                        \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                         \
        resident_iso_kernel<m, n><<<dim3((unsigned)planes), kNT, lds, s>>>(hty, s_in, s_out, fmap, q, x_out, Ct, \
                                                                            twM, twN, prm, k, K);                \
        return 0;                                                                                                \
    }
    RS_SHAPES(X)
#undef X
    return -1;
}

int launch(int M, int N, size_t planes, hipStream_t s, const float* hty, float* sA, float* sB, float* traj,
           size_t traj_stride, float* x_out, const float* Ct, const float2* twM, const float2* twN, const float* prm,
           int maxit) {
#define X(m, n)                                                                                                  \
    if (M == m && N == n) {                                                                                      \
        constexpr size_t lds = Geo<m, n>::lds_bytes();                                                           \
        (void)hipFuncSetAttribute((const void*)resident_kernel<m, n>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                  (int)lds);                                                                     \
        resident_kernel<m, n><<<dim3((unsigned)planes), kNT, lds, s>>>(hty, sA, sB, traj, traj_stride, x_out, Ct, \
                                                                        twM, twN, prm, maxit);                   \
        return 0;                                                                                                \
    }
    RS_SHAPES(X)
#undef X
    return -1;
}

}  // namespace rs
}  // namespace admm
