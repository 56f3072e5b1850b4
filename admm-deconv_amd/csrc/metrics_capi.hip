// metrics_capi.hip -- the image-quality losses / metrics that follow the solver in every training
// step of the reference, as HIP kernels behind the C ABI:
//   GMSD  src/metrics/gmsd.jl:13-27 (+ imgrads / gradientsmag, src/metrics/iqa_utils.jl:24-55):
//         the training loss (src/train.jl:129,191)
//   SSIM  src/metrics/ssim.jl:84-124 (ssim_loss :148, ssim_loss_fast :160): the demo's loss
//         (src/ADMM_Deconv.jl:31)
//   per-image MSE for peak_snr (src/metrics/psnr.jl:5-10) and Flux.mse (src/train.jl:131)
// Layout as the solver: Julia (M, N, C, B) == C float[B][C][N][M]; statistics per image over dims
// 1..3 (M, N, C).  All three are HBM-bound stencils + reductions (no MFMA): each kernel reads its
// inputs once through an LDS tile with halo and writes one partial sum per block (reduced in a fixed
// order: deterministic).  Gradients are w.r.t. the first argument x, weighted per image by the
// upstream gradient of the per-image value (NULL = d mean / d value = 1/B).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "../../include/admm_deconv.h"
#include "../../include/admm_metrics.h"

namespace admm_internal {
int fail_msg(int code, const char* msg);   // admm_capi.hip (sets admm_last_error)
}

namespace admm {
namespace metrics {

constexpr int kT = 256;          // threads per block
constexpr int TX = 64, TY = 16;  // output tile (dim1 x dim2)
constexpr int kMaxTaps = 15;

struct Taps {
    float k[kMaxTaps];
    int n;
};

// circular index (any offset); in range -- the common case -- it is one compare, not two integer divisions
__device__ __forceinline__ int wrapc(int i, int n) {
    if ((unsigned)i < (unsigned)n) return i;
    return ((i % n) + n) % n;
}
// NNlib pad_symmetric: ... b a | a b c | c b ...
__device__ __forceinline__ int mirror(int i, int n) { return i < 0 ? -i - 1 : (i >= n ? 2 * n - i - 1 : i); }

__device__ __forceinline__ void block_sum_d2(double a, double b, double* out) {
    __shared__ double red[2 * (kT / 64)];
    for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_down(a, off);
        b += __shfl_down(b, off);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[2 * w] = a;
        red[2 * w + 1] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double sa = 0.0, sb = 0.0;
        for (int i = 0; i < kT / 64; ++i) {
            sa += red[2 * i];
            sb += red[2 * i + 1];
        }
        out[0] = sa;
        out[1] = sb;
    }
}

// ---------------------------------------------------------------------------------------------
// SSIM.  Window statistics by a separable kernel k (ssim_kernel = k k^T, ssim.jl:23-31):
//   mu_x = k * x, sigma_x^2 = k * x^2 - mu_x^2, sigma_xy = k * (x y) - mu_x mu_y   (valid conv when
//   crop, else same-size on the symmetric padding, ssim.jl:103-108)
//   S = (2 mu_x mu_y + C1)(2 sigma_xy + C2) / ((mu_x^2 + mu_y^2 + C1)(sigma_x^2 + sigma_y^2 + C2))
// GRAD also stores, per valid output q, w dS/d(mu_x) - 2 mu_x w dS/d(sx2) - mu_y w dS/d(sxy), w dS/d(sx2)
// and w dS/d(sxy) (w = upstream / (Mo No C)): x_bar = k^T * A + 2 x (k^T * B) + y (k^T * C).
// ---------------------------------------------------------------------------------------------
template <bool GRAD>
__global__ __launch_bounds__(kT) void ssim_fwd_kernel(const float* __restrict__ x, const float* __restrict__ y, int M,
                                                      int N, int Mo, int No, Taps tp, int crop, float C1, float C2,
                                                      double* __restrict__ part, float* __restrict__ coef,
                                                      const float* __restrict__ wimg, int C, float wdef) {
    const int ks = tp.n;
    const int IX = TX + ks - 1, IY = TY + ks - 1;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float* xs = reinterpret_cast<float*>(smem_raw);
    float* ys = xs + IX * IY;
    float* hs = ys + IX * IY;   // 5 x IY x TX
    const int plane = blockIdx.z;
    const int i0 = blockIdx.x * TX, j0 = blockIdx.y * TY;
    const size_t MN = (size_t)M * N;
    const float* xp = x + plane * MN;
    const float* yp = y + plane * MN;
    const int pad = (ks - 1 + 1) / 2;   // cld(ks - 1, 2) (Flux calc_padding, ssim.jl:101)
    for (int idx = threadIdx.x; idx < IX * IY; idx += kT) {
        const int jj = idx / IX, ii = idx - jj * IX;
        int gi = i0 + ii, gj = j0 + jj;
        float xv = 0.f, yv = 0.f;
        if (crop) {
            if (gi < M && gj < N) {
                xv = xp[(size_t)gj * M + gi];
                yv = yp[(size_t)gj * M + gi];
            }
        } else {
            gi = mirror(gi - pad, M);
            gj = mirror(gj - pad, N);
            if (gi >= 0 && gi < M && gj >= 0 && gj < N) {
                xv = xp[(size_t)gj * M + gi];
                yv = yp[(size_t)gj * M + gi];
            }
        }
        xs[idx] = xv;
        ys[idx] = yv;
    }
    __syncthreads();
    const int HS = IY * TX;
    for (int idx = threadIdx.x; idx < HS; idx += kT) {
        const int r = idx / TX, o = idx - r * TX;
        float a = 0.f, b = 0.f, aa = 0.f, bb = 0.f, ab = 0.f;
        for (int t = 0; t < ks; ++t) {
            const float w = tp.k[t];
            const float xv = xs[r * IX + o + t], yv = ys[r * IX + o + t];
            a = fmaf(w, xv, a);
            b = fmaf(w, yv, b);
            aa = fmaf(w, xv * xv, aa);
            bb = fmaf(w, yv * yv, bb);
            ab = fmaf(w, xv * yv, ab);
        }
        hs[idx] = a;
        hs[HS + idx] = b;
        hs[2 * HS + idx] = aa;
        hs[3 * HS + idx] = bb;
        hs[4 * HS + idx] = ab;
    }
    __syncthreads();
    const int b_img = plane / C;
    const float w = GRAD ? (wimg ? wimg[b_img] : wdef) / ((float)Mo * (float)No * (float)C) : 0.f;
    double acc = 0.0;
    for (int idx = threadIdx.x; idx < TX * TY; idx += kT) {
        const int oj = idx / TX, oi = idx - oj * TX;
        const int qi = i0 + oi, qj = j0 + oj;
        if (qi >= Mo || qj >= No) continue;
        float mx = 0.f, my = 0.f, exx = 0.f, eyy = 0.f, exy = 0.f;
        for (int t = 0; t < ks; ++t) {
            const float kw = tp.k[t];
            const int o = (oj + t) * TX + oi;
            mx = fmaf(kw, hs[o], mx);
            my = fmaf(kw, hs[HS + o], my);
            exx = fmaf(kw, hs[2 * HS + o], exx);
            eyy = fmaf(kw, hs[3 * HS + o], eyy);
            exy = fmaf(kw, hs[4 * HS + o], exy);
        }
        const float mx2 = mx * mx, my2 = my * my, mxy = mx * my;
        const float sx = exx - mx2, sy = eyy - my2, sxy = exy - mxy;
        const float n1 = 2.f * mxy + C1, n2 = 2.f * sxy + C2;
        const float d1 = mx2 + my2 + C1, d2 = sx + sy + C2;
        const float S = (n1 * n2) / (d1 * d2);
        acc += (double)S;
        if constexpr (GRAD) {
            const float dmu = 2.f * my * n2 / (d1 * d2) - 2.f * mx * S / d1;   // dS/d mu_x
            const float dsx = -S / d2;                                          // dS/d sigma_x^2
            const float dsxy = 2.f * n1 / (d1 * d2);                            // dS/d sigma_xy
            const size_t q = (size_t)plane * Mo * No + (size_t)qj * Mo + qi;
            const size_t P = (size_t)gridDim.z * Mo * No;
            coef[q] = w * (dmu - 2.f * mx * dsx - my * dsxy);
            coef[P + q] = w * dsx;
            coef[2 * P + q] = w * dsxy;
        }
    }
    block_sum_d2(acc, 0.0, part + 2 * ((size_t)plane * gridDim.x * gridDim.y + blockIdx.y * gridDim.x + blockIdx.x));
}

// x_bar = k^T * A + 2 x (k^T * B) + y (k^T * C) over the full plane (maps zero outside the valid range)
__global__ __launch_bounds__(kT) void ssim_bwd_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                      const float* __restrict__ coef, float* __restrict__ xbar, int M,
                                                      int N, int Mo, int No, Taps tp, int planes) {
    const int ks = tp.n;
    const int IX = TX + ks - 1, IY = TY + ks - 1;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float* cs = reinterpret_cast<float*>(smem_raw);   // 3 x IY x IX
    float* hs = cs + 3 * IX * IY;                      // 3 x IY x TX
    const int plane = blockIdx.z;
    const int i0 = blockIdx.x * TX, j0 = blockIdx.y * TY;
    const size_t P = (size_t)planes * Mo * No;
    const float* cp = coef + (size_t)plane * Mo * No;
    for (int idx = threadIdx.x; idx < IX * IY; idx += kT) {
        const int jj = idx / IX, ii = idx - jj * IX;
        const int qi = i0 - (ks - 1) + ii, qj = j0 - (ks - 1) + jj;
        const bool in = qi >= 0 && qi < Mo && qj >= 0 && qj < No;
        const size_t q = (size_t)qj * Mo + qi;
        cs[idx] = in ? cp[q] : 0.f;
        cs[IX * IY + idx] = in ? cp[P + q] : 0.f;
        cs[2 * IX * IY + idx] = in ? cp[2 * P + q] : 0.f;
    }
    __syncthreads();
    const int HS = IY * TX;
    for (int idx = threadIdx.x; idx < HS; idx += kT) {
        const int r = idx / TX, o = idx - r * TX;
        float a = 0.f, b = 0.f, c = 0.f;
        for (int t = 0; t < ks; ++t) {
            const float w = tp.k[t];
            const int s = r * IX + o + (ks - 1) - t;
            a = fmaf(w, cs[s], a);
            b = fmaf(w, cs[IX * IY + s], b);
            c = fmaf(w, cs[2 * IX * IY + s], c);
        }
        hs[idx] = a;
        hs[HS + idx] = b;
        hs[2 * HS + idx] = c;
    }
    __syncthreads();
    const size_t MN = (size_t)M * N;
    for (int idx = threadIdx.x; idx < TX * TY; idx += kT) {
        const int oj = idx / TX, oi = idx - oj * TX;
        const int pi = i0 + oi, pj = j0 + oj;
        if (pi >= M || pj >= N) continue;
        float a = 0.f, b = 0.f, c = 0.f;
        for (int t = 0; t < ks; ++t) {
            const float w = tp.k[t];
            const int o = (oj + (ks - 1) - t) * TX + oi;
            a = fmaf(w, hs[o], a);
            b = fmaf(w, hs[HS + o], b);
            c = fmaf(w, hs[2 * HS + o], c);
        }
        const size_t p = plane * MN + (size_t)pj * M + pi;
        xbar[p] = a + 2.f * x[p] * b + y[p] * c;
    }
}

// ---------------------------------------------------------------------------------------------
// GMSD.  Sobel gradients on the circular padding (iqa_utils.jl:24-50; Kx[a][b] = c_a w_b / 8 with
// c = (1, 0, -1) along dim 1, w = (1, 2, 1) along dim 2; Ky = Kx^T -- correlation or convolution
// differ only in sign, which the magnitude removes), m = sqrt(gx^2 + gy^2 + 1e-16) (:53-55),
// gms = ((2 - a) m_x m_y + t) / (m_x^2 + m_y^2 - a m_x m_y + t) (gmsd.jl:5-10), per image
// gmsd = sqrt(mean((gms - mean gms)^2)) over M, N, C (gmsd.jl:23-25).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void sobel(const float* s, int W, int r, int c, float& gx, float& gy) {
    // s: LDS tile of width W; (r, c) the centre.  gx: derivative along dim 1 (columns c), smoothing
    // along dim 2 (rows r)
    const float a00 = s[(r - 1) * W + c - 1], a01 = s[(r - 1) * W + c], a02 = s[(r - 1) * W + c + 1];
    const float a10 = s[r * W + c - 1], a12 = s[r * W + c + 1];
    const float a20 = s[(r + 1) * W + c - 1], a21 = s[(r + 1) * W + c], a22 = s[(r + 1) * W + c + 1];
    gx = ((a00 - a02) + 2.f * (a10 - a12) + (a20 - a22)) * 0.125f;
    gy = ((a00 - a20) + 2.f * (a01 - a21) + (a02 - a22)) * 0.125f;
}

// The hardware square root and reciprocal (1 ulp each, v_sqrt_f32 / v_rcp_f32) instead of the correctly rounded
// sequences: den >= t > 0 and m >= 1e-8 are normal numbers, and the loss is held to 2e-5 of the fp64 oracle
// (tests/test_gpu_metrics.py).
__device__ __forceinline__ float gms_val(float mx, float my, float t, float al, float& dgdmx) {
    const float num = (2.f - al) * mx * my + t;
    const float den = mx * mx + my * my - al * mx * my + t;
    const float r = __builtin_amdgcn_rcpf(den);
    dgdmx = ((2.f - al) * my * den - num * (2.f * mx - al * my)) * (r * r);
    return num * r;
}
__device__ __forceinline__ float gmag(float gx, float gy) { return __builtin_amdgcn_sqrtf(gx * gx + gy * gy + 1e-16f); }

// per-block (sum gms, sum gms^2).  (256 x 16 tiles -- 1.02x halo reads instead of 1.16x, 16 outputs per thread --
// measured slower at c5's 960 planes of 256^2: forward 245 -> 260 us, backward 400 -> 568 us; not kept)
__global__ __launch_bounds__(kT) void gmsd_fwd_kernel(const float* __restrict__ x, const float* __restrict__ y, int M,
                                                      int N, float t, float al, double* __restrict__ part) {
    constexpr int W = TX + 2, Hh = TY + 2;
    __shared__ float xs[W * Hh], ys[W * Hh];
    const int plane = blockIdx.z;
    const int i0 = blockIdx.x * TX, j0 = blockIdx.y * TY;
    const size_t MN = (size_t)M * N;
    const float* xp = x + plane * MN;
    const float* yp = y + plane * MN;
    for (int idx = threadIdx.x; idx < W * Hh; idx += kT) {
        const int r = idx / W, c = idx - r * W;
        const size_t o = (size_t)wrapc(j0 + r - 1, N) * M + wrapc(i0 + c - 1, M);
        xs[idx] = xp[o];
        ys[idx] = yp[o];
    }
    __syncthreads();
    double s1 = 0.0, s2 = 0.0;
    for (int idx = threadIdx.x; idx < TX * TY; idx += kT) {
        const int r = idx / TX, c = idx - r * TX;
        if (i0 + c >= M || j0 + r >= N) continue;
        float gx, gy, hx, hy, dd;
        sobel(xs, W, r + 1, c + 1, gx, gy);
        sobel(ys, W, r + 1, c + 1, hx, hy);
        const float mx = gmag(gx, gy), my = gmag(hx, hy);
        const float g = gms_val(mx, my, t, al, dd);
        s1 += g;
        s2 += (double)g * g;
    }
    block_sum_d2(s1, s2, part + 2 * ((size_t)plane * gridDim.x * gridDim.y + blockIdx.y * gridDim.x + blockIdx.x));
}

// x_bar(p) = sum_{a,b} Kx[a][b] gbx(p - (a-1, b-1)) + Ky[a][b] gby(...),  gb = coef (g - mu) dg/dmx (gx, gy)/mx
__global__ __launch_bounds__(kT) void gmsd_bwd_kernel(const float* __restrict__ x, const float* __restrict__ y, int M,
                                                      int N, float t, float al, const float* __restrict__ stats, int C,
                                                      float* __restrict__ xbar) {
    constexpr int W = TX + 4, Hh = TY + 4, W1 = TX + 2, H1 = TY + 2;
    __shared__ float xs[W * Hh], ys[W * Hh], gbx[W1 * H1], gby[W1 * H1];
    const int plane = blockIdx.z;
    const int i0 = blockIdx.x * TX, j0 = blockIdx.y * TY;
    const size_t MN = (size_t)M * N;
    const float* xp = x + plane * MN;
    const float* yp = y + plane * MN;
    const int b = plane / C;
    const float mu = stats[2 * b], cf = stats[2 * b + 1];
    for (int idx = threadIdx.x; idx < W * Hh; idx += kT) {
        const int r = idx / W, c = idx - r * W;
        const size_t o = (size_t)wrapc(j0 + r - 2, N) * M + wrapc(i0 + c - 2, M);
        xs[idx] = xp[o];
        ys[idx] = yp[o];
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < W1 * H1; idx += kT) {
        const int r = idx / W1, c = idx - r * W1;
        float gx, gy, hx, hy, dg;
        sobel(xs, W, r + 1, c + 1, gx, gy);
        sobel(ys, W, r + 1, c + 1, hx, hy);
        const float mx = gmag(gx, gy), my = gmag(hx, hy);
        const float g = gms_val(mx, my, t, al, dg);
        const float gm = cf * (g - mu) * dg * __builtin_amdgcn_rcpf(mx);
        gbx[idx] = gm * gx;
        gby[idx] = gm * gy;
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < TX * TY; idx += kT) {
        const int r = idx / TX, c = idx - r * TX;
        const int pi = i0 + c, pj = j0 + r;
        if (pi >= M || pj >= N) continue;
        // centre (r + 1, c + 1) of the gb tile; p - (a-1, b-1): column c + 1 - (a - 1), row r + 1 - (b - 1)
        const int R = r + 1, Cc = c + 1;
        const float* X = gbx;
        const float* Y = gby;
        // Kx[a][b] = c_a w_b / 8: a along dim 1 (columns), b along dim 2 (rows); Ky[a][b] = c_b w_a / 8
        float acc = 0.f;
#pragma unroll
        for (int bb = 0; bb < 3; ++bb) {
#pragma unroll
            for (int aa = 0; aa < 3; ++aa) {
                const float ca = aa == 0 ? 1.f : (aa == 2 ? -1.f : 0.f), cb = bb == 0 ? 1.f : (bb == 2 ? -1.f : 0.f);
                const float wa = aa == 1 ? 2.f : 1.f, wb = bb == 1 ? 2.f : 1.f;
                const int o = (R - (bb - 1)) * W1 + (Cc - (aa - 1));
                acc += 0.125f * (ca * wb * X[o] + cb * wa * Y[o]);
            }
        }
        xbar[plane * MN + (size_t)pj * M + pi] = acc;
    }
}

// per-block sum of (x - y)^2
__global__ __launch_bounds__(kT) void sqerr_kernel(const float* __restrict__ x, const float* __restrict__ y, size_t MN,
                                                   int nblk, double* __restrict__ part) {
    const int plane = blockIdx.y;
    const float* xp = x + plane * MN;
    const float* yp = y + plane * MN;
    double acc = 0.0;
    for (size_t q = (size_t)blockIdx.x * kT + threadIdx.x; q < MN; q += (size_t)nblk * kT) {
        const float d = xp[q] - yp[q];
        acc += (double)d * d;
    }
    block_sum_d2(acc, 0.0, part + 2 * ((size_t)plane * nblk + blockIdx.x));
}

// per image (one block each): sum the C * nblk partial pairs in a fixed order (thread t the strided
// subset t, t + kT, ..., then the block's fixed-order tree).
//   mode 0 (SSIM, MSE): out[b] = s1 / count
//   mode 1 (GMSD): mu = s1/count, var = s2/count - mu^2, out[b] = sqrt(var); stats[b] = (mu, w_b / (count sqrt(var)))
__global__ __launch_bounds__(kT) void reduce_img_kernel(const double* __restrict__ part, int per_img, double count,
                                                        int mode, float* __restrict__ out, float* __restrict__ stats,
                                                        const float* __restrict__ wimg, float wdef, int B) {
    const int b = blockIdx.x;
    __shared__ double tot[2];
    double a = 0.0, c = 0.0;
    const double* p = part + 2 * (size_t)b * per_img;
    for (int i = threadIdx.x; i < per_img; i += kT) {
        a += p[2 * i];
        c += p[2 * i + 1];
    }
    block_sum_d2(a, c, tot);
    __syncthreads();
    if (threadIdx.x != 0) return;
    const double s1 = tot[0], s2 = tot[1];
    if (mode == 0) {
        out[b] = (float)(s1 / count);
        return;
    }
    const double mu = s1 / count;
    double var = s2 / count - mu * mu;
    var = var > 0.0 ? var : 0.0;
    out[b] = (float)sqrt(var);
    if (stats) {
        const float w = wimg ? wimg[b] : wdef;
        stats[2 * b] = (float)mu;
        stats[2 * b + 1] = (float)(w / (count * sqrt(var)));
    }
}

}  // namespace metrics
}  // namespace admm

namespace {

using namespace admm::metrics;

size_t align256(size_t v) { return (v + 255) & ~size_t(255); }

struct MLayout {
    size_t part, stats, coef, total;
    int nblk;
};

MLayout mlayout(int M, int N, int C, int B, int ks, bool grad) {
    MLayout L{};
    const size_t planes = (size_t)C * B;
    const int bx = (M + TX - 1) / TX, by = (N + TY - 1) / TY;
    L.nblk = bx * by;
    size_t off = 0;
    L.part = off;
    off = align256(off + planes * (size_t)(L.nblk > 64 ? L.nblk : 64) * 16);
    L.stats = off;
    off = align256(off + (size_t)B * 12);   // (mu, coefficient) per image + the backward's scratch copy of out
    L.coef = off;
    if (grad && ks > 0) off = align256(off + 3 * planes * (size_t)M * N * 4);
    L.total = off;
    return L;
}

int check_common(const float* x, const float* y, int M, int N, int C, int B, float* out, void* ws, size_t ws_bytes,
                 size_t need) {
    if (!x || !y || !out) return admm_internal::fail_msg(ADMM_E_INVALID, "x, y and out must be device pointers");
    if (M < 1 || N < 1 || C < 1 || B < 1) return admm_internal::fail_msg(ADMM_E_INVALID, "sizes must be positive");
    if ((size_t)C * B > 65535) return admm_internal::fail_msg(ADMM_E_UNSUPPORTED, "at most 65535 planes per call");
    if (!ws || ws_bytes < need || (reinterpret_cast<uintptr_t>(ws) & 255))
        return admm_internal::fail_msg(ADMM_E_WORKSPACE, "metrics workspace too small or not 256-byte aligned");
    return ADMM_OK;
}

int launched() {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return admm_internal::fail_msg(ADMM_E_HIP, hipGetErrorString(e));
    return ADMM_OK;
}

}  // namespace

extern "C" {

int admm_metrics_workspace_bytes(int M, int N, int C, int B, int ks, int grad, size_t* out_bytes) {
    if (!out_bytes) return admm_internal::fail_msg(ADMM_E_INVALID, "out_bytes is NULL");
    *out_bytes = mlayout(M, N, C, B, ks, grad != 0).total;
    return ADMM_OK;
}

dim3 gmsd_grid(int M, int N, int planes) { return dim3((M + TX - 1) / TX, (N + TY - 1) / TY, (unsigned)planes); }
void launch_gmsd_fwd(const float* x, const float* y, int M, int N, int planes, float t, float al, double* part,
                     hipStream_t s) {
    hipLaunchKernelGGL(gmsd_fwd_kernel, gmsd_grid(M, N, planes), dim3(kT), 0, s, x, y, M, N, t, al, part);
}
void launch_gmsd_bwd(const float* x, const float* y, int M, int N, int C, int planes, float t, float al,
                     const float* stats, float* xbar, hipStream_t s) {
    hipLaunchKernelGGL(gmsd_bwd_kernel, gmsd_grid(M, N, planes), dim3(kT), 0, s, x, y, M, N, t, al, stats, C, xbar);
}
int gmsd_blocks(int M, int N) { return ((M + TX - 1) / TX) * ((N + TY - 1) / TY); }

int admm_gmsd_f32(const float* x, const float* y, int M, int N, int C, int B, float t, float alpha, float* out,
                  const float* out_bar, float* x_bar, void* ws, size_t ws_bytes, void* stream) {
    const MLayout L = mlayout(M, N, C, B, 0, x_bar != nullptr);
    int rc = check_common(x, y, M, N, C, B, out, ws, ws_bytes, L.total);
    if (rc) return rc;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    unsigned char* w = static_cast<unsigned char*>(ws);
    double* part = reinterpret_cast<double*>(w + L.part);
    float* stats = reinterpret_cast<float*>(w + L.stats);
    launch_gmsd_fwd(x, y, M, N, C * B, t, alpha, part, s);
    if ((rc = launched())) return rc;
    hipLaunchKernelGGL(reduce_img_kernel, dim3(B), dim3(kT), 0, s, part, C * gmsd_blocks(M, N),
                       (double)M * N * C, 1, out, x_bar ? stats : nullptr, out_bar, 1.0f / B, B);
    if ((rc = launched())) return rc;
    if (x_bar) {
        launch_gmsd_bwd(x, y, M, N, C, C * B, t, alpha, stats, x_bar, s);
        if ((rc = launched())) return rc;
    }
    return ADMM_OK;
}

int admm_gmsd_backward_f32(const float* x, const float* y, int M, int N, int C, int B, float t, float alpha,
                           const float* out_bar, float* x_bar, void* ws, size_t ws_bytes, void* stream) {
    const MLayout L = mlayout(M, N, C, B, 0, true);
    if (!x_bar) return admm_internal::fail_msg(ADMM_E_INVALID, "x_bar must be a device pointer");
    int rc = check_common(x, y, M, N, C, B, x_bar, ws, ws_bytes, L.total);
    if (rc) return rc;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    unsigned char* w = static_cast<unsigned char*>(ws);
    const double* part = reinterpret_cast<const double*>(w + L.part);   // the forward's partial sums
    float* stats = reinterpret_cast<float*>(w + L.stats);
    // the per-image figure is not wanted again: the reduction writes it into the stats slot's tail-free scratch
    float* out = reinterpret_cast<float*>(w + L.stats) + 2 * B;
    hipLaunchKernelGGL(reduce_img_kernel, dim3(B), dim3(kT), 0, s, part, C * gmsd_blocks(M, N), (double)M * N * C, 1,
                       out, stats, out_bar, 1.0f / B, B);
    if ((rc = launched())) return rc;
    launch_gmsd_bwd(x, y, M, N, C, C * B, t, alpha, stats, x_bar, s);
    return launched();
}

int admm_ssim_f32(const float* x, const float* y, int M, int N, int C, int B, const float* taps, int ks, float peakval,
                  int crop, float* out, const float* out_bar, float* x_bar, void* ws, size_t ws_bytes, void* stream) {
    if (!taps || ks < 1 || ks > kMaxTaps)
        return admm_internal::fail_msg(ADMM_E_INVALID, "ssim kernel: 1..15 separable taps (host pointer) required");
    if (crop && (M < ks || N < ks)) return admm_internal::fail_msg(ADMM_E_INVALID, "image smaller than the SSIM window");
    if (x_bar && !crop)
        return admm_internal::fail_msg(ADMM_E_UNSUPPORTED, "SSIM gradient implemented for crop=true (the reference default)");
    const MLayout L = mlayout(M, N, C, B, ks, x_bar != nullptr);
    int rc = check_common(x, y, M, N, C, B, out, ws, ws_bytes, L.total);
    if (rc) return rc;
    Taps tp{};
    tp.n = ks;
    for (int i = 0; i < ks; ++i) tp.k[i] = taps[i];
    const int Mo = crop ? M - ks + 1 : M, No = crop ? N - ks + 1 : N;
    const float C1 = (peakval * 0.01f) * (peakval * 0.01f), C2 = (peakval * 0.03f) * (peakval * 0.03f);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    unsigned char* w = static_cast<unsigned char*>(ws);
    double* part = reinterpret_cast<double*>(w + L.part);
    float* coef = reinterpret_cast<float*>(w + L.coef);
    const dim3 g((Mo + TX - 1) / TX, (No + TY - 1) / TY, (unsigned)(C * B));
    const int IX = TX + ks - 1, IY = TY + ks - 1;
    const size_t lds = (size_t)(2 * IX * IY + 5 * IY * TX) * 4;
    if (x_bar) {
        hipLaunchKernelGGL(ssim_fwd_kernel<true>, g, dim3(kT), lds, s, x, y, M, N, Mo, No, tp, crop, C1, C2, part, coef,
                           out_bar, C, 1.0f / B);
    } else {
        hipLaunchKernelGGL(ssim_fwd_kernel<false>, g, dim3(kT), lds, s, x, y, M, N, Mo, No, tp, crop, C1, C2, part,
                           coef, out_bar, C, 1.0f / B);
    }
    if ((rc = launched())) return rc;
    hipLaunchKernelGGL(reduce_img_kernel, dim3(B), dim3(kT), 0, s, part, C * (int)(g.x * g.y),
                       (double)Mo * No * C, 0, out, nullptr, nullptr, 0.0f, B);
    if ((rc = launched())) return rc;
    if (x_bar) {
        const dim3 gb((M + TX - 1) / TX, (N + TY - 1) / TY, (unsigned)(C * B));
        const size_t lb = (size_t)(3 * IX * IY + 3 * IY * TX) * 4;
        hipLaunchKernelGGL(ssim_bwd_kernel, gb, dim3(kT), lb, s, x, y, coef, x_bar, M, N, Mo, No, tp, C * B);
        if ((rc = launched())) return rc;
    }
    return ADMM_OK;
}

int admm_mse_f32(const float* x, const float* y, int M, int N, int C, int B, float* out, void* ws, size_t ws_bytes,
                 void* stream) {
    const MLayout L = mlayout(M, N, C, B, 0, false);
    int rc = check_common(x, y, M, N, C, B, out, ws, ws_bytes, L.total);
    if (rc) return rc;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    double* part = reinterpret_cast<double*>(static_cast<unsigned char*>(ws) + L.part);
    const size_t MN = (size_t)M * N;
    int nblk = (int)((MN + kT * 8 - 1) / (kT * 8));
    nblk = nblk < 1 ? 1 : (nblk > 64 ? 64 : nblk);
    hipLaunchKernelGGL(sqerr_kernel, dim3(nblk, C * B), dim3(kT), 0, s, x, y, MN, nblk, part);
    if ((rc = launched())) return rc;
    hipLaunchKernelGGL(reduce_img_kernel, dim3(B), dim3(kT), 0, s, part, C * nblk, (double)MN * C, 0, out,
                       nullptr, nullptr, 0.0f, B);
    return launched();
}

}  // extern "C"
