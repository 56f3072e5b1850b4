/*
 * admm_metrics.h -- C ABI of the image-quality losses / metrics that follow the solver in every
 * training step of the reference: GMSD (src/metrics/gmsd.jl:13-27, the training
 * loss, src/train.jl:129,191), SSIM (src/metrics/ssim.jl:84-124, ssim_loss :148, ssim_loss_fast
 * :160) and the per-image MSE behind peak_snr (src/metrics/psnr.jl:5-10) and Flux.mse.
 *
 * Conventions as admm_deconv.h: device pointers, layout Julia (M, N, C, B) == C float[B][C][N][M],
 * caller-owned workspace (admm_metrics_workspace_bytes, 256-byte aligned), asynchronous on `stream`,
 * 0 or a negative ADMM_E_* code (admm_last_error() has the message).  Deterministic.
 * Outputs are PER IMAGE (statistics over M, N, C): out[b], b < B.  With x_bar != NULL the call also
 * writes x_bar = sum_b out_bar[b] d out[b] / dx (out_bar: device, B floats; NULL means 1/B each,
 * i.e. the gradient of the batch mean the reference reduces with).  No gradient w.r.t. y.
 */
#ifndef ADMM_METRICS_H
#define ADMM_METRICS_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ks: SSIM window taps (0 for GMSD / MSE); grad: whether x_bar will be requested. */
int admm_metrics_workspace_bytes(int M, int N, int C, int B, int ks, int grad, size_t* out_bytes);

/* GMSD per image: Sobel gradient magnitudes on the circular padding (iqa_utils.jl:24-55),
 * gms = ((2-alpha) m_x m_y + t) / (m_x^2 + m_y^2 - alpha m_x m_y + t), out[b] = std over the image of
 * gms (gmsd.jl:23-25).  Reference defaults t = 0.0026, alpha = 0. */
int admm_gmsd_f32(const float* x, const float* y, int M, int N, int C, int B, float t, float alpha,
                  float* out, const float* out_bar, float* x_bar, void* workspace,
                  size_t workspace_bytes, void* stream);

/* The GMSD gradient without re-running the forward: `workspace` must hold what a preceding admm_gmsd_f32 call
 * left there for the same x, y, sizes, t and alpha (its per-block partial sums; enqueued before this call on the
 * same stream or ordered with it), and be at least admm_metrics_workspace_bytes(M, N, C, B, 0, 1) bytes.  x_bar
 * = d(sum_b out_bar[b] out[b]) / dx (out_bar NULL: 1/B each, the mean). */
int admm_gmsd_backward_f32(const float* x, const float* y, int M, int N, int C, int B, float t, float alpha,
                           const float* out_bar, float* x_bar, void* workspace, size_t workspace_bytes,
                           void* stream);

/* SSIM per image: mean of the SSIM map with the separable window taps[0..ks) (host pointer, ks <= 15;
 * the reference's 11-tap Gaussian or a box), C1 = (0.01 peakval)^2, C2 = (0.03 peakval)^2; crop != 0:
 * valid window positions, else same-size on the symmetric padding (ssim.jl:99-108).  x_bar needs
 * crop != 0. */
int admm_ssim_f32(const float* x, const float* y, int M, int N, int C, int B, const float* taps, int ks,
                  float peakval, int crop, float* out, const float* out_bar, float* x_bar,
                  void* workspace, size_t workspace_bytes, void* stream);

/* mean squared error per image (over M, N, C). */
int admm_mse_f32(const float* x, const float* y, int M, int N, int C, int B, float* out, void* workspace,
                 size_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* ADMM_METRICS_H */
