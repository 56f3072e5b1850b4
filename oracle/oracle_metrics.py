"""CPU oracle for the image-quality metrics -- TEST INFRASTRUCTURE ONLY.

numpy restatement (fp64) of the reference's src/metrics/ functions that follow the solver in the
training step: `gmsd` (gmsd.jl:13-27 with imgrads / gradientsmag, iqa_utils.jl:24-55), `ssim`
(ssim.jl:84-124; ssim_kernel :23-38) and `peak_snr` (psnr.jl:5-10).  Only tests/ may import it.

Arrays are Julia-order (M, N, C, B) (see oracle_np.from_c / to_c).  NNlib `conv` is a true
convolution (the kernel is flipped); both are restated literally here (the SSIM window is symmetric,
and the Sobel flip only changes the sign of the gradients).  Parity unpinned against Julia itself
(absent): these follow the reference's formulas line by line.
"""
from __future__ import annotations

import numpy as np
from numpy.lib.stride_tricks import sliding_window_view

SSIM_KERNEL = np.array([0.00102838008447911, 0.007598758135239185, 0.03600077212843083, 0.10936068950970002,
                        0.2130055377112537, 0.26601172486179436, 0.2130055377112537, 0.10936068950970002,
                        0.03600077212843083, 0.007598758135239185, 0.00102838008447911])   # ssim.jl:6-17

# iqa_utils.jl:12-17: cat([1,0,-1],[2,0,-2],[1,0,-1], dims=2) ./ 8  -> K[a, b] (a along dim 1)
SOBEL_KERNEL_X = np.stack([np.array([1.0, 0.0, -1.0]), np.array([2.0, 0.0, -2.0]), np.array([1.0, 0.0, -1.0])],
                          axis=1) / 8.0
SOBEL_KERNEL_Y = SOBEL_KERNEL_X.T.copy()


def conv2_valid(x, K):
    """NNlib.conv (flipped kernel) of every (M, N) plane of x (M, N, C, B) with K (ka, kb), valid size."""
    Kf = K[::-1, ::-1]
    win = sliding_window_view(x, K.shape, axis=(0, 1))        # (M-ka+1, N-kb+1, C, B, ka, kb)
    return np.einsum("ijcbuv,uv->ijcb", win, Kf)


def ssim(x, y, kernel=None, peakval=1.0, crop=True):
    """ssim.jl:84-124 -- returns (mean over images, per-image values)."""
    k = SSIM_KERNEL if kernel is None else np.asarray(kernel, np.float64)
    K = np.outer(k, k)                                         # ssim_kernel for 4-D input (ssim.jl:27)
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    C1, C2 = (peakval * 0.01) ** 2, (peakval * 0.03) ** 2      # ssim.jl:96-97
    if not crop:                                               # ssim.jl:99-108: pad_symmetric
        lo, hi = -(-(len(k) - 1) // 2), (len(k) - 1) // 2
        pw = ((lo, hi), (lo, hi), (0, 0), (0, 0))
        x = np.pad(x, pw, mode="symmetric")
        y = np.pad(y, pw, mode="symmetric")
    mx = conv2_valid(x, K)
    my = conv2_valid(y, K)
    mx2, my2, mxy = mx ** 2, my ** 2, mx * my
    sx = conv2_valid(x ** 2, K) - mx2
    sy = conv2_valid(y ** 2, K) - my2
    sxy = conv2_valid(x * y, K) - mxy
    smap = (2 * mxy + C1) * (2 * sxy + C2) / ((mx2 + my2 + C1) * (sx + sy + C2))
    per = smap.mean(axis=(0, 1, 2))                            # ims_ssim = mean(ssim_map, dims=(1,2,3))
    return per.mean(), per


def imgrads(x):
    """iqa_utils.jl:24-50: Sobel gradients of pad_circular(x, 1), grouped per channel."""
    xp = np.pad(np.asarray(x, np.float64), ((1, 1), (1, 1), (0, 0), (0, 0)), mode="wrap")
    return conv2_valid(xp, SOBEL_KERNEL_X), conv2_valid(xp, SOBEL_KERNEL_Y)


def gmsd(x, y, t=0.0026, alpha=0.0):
    """gmsd.jl:13-27 with reduction = mean -- returns (mean over images, per-image values)."""
    gx, gy = imgrads(x)
    hx, hy = imgrads(y)
    mx = np.sqrt(gx ** 2 + gy ** 2 + 1e-16)                    # gradientsmag, iqa_utils.jl:53-55
    my = np.sqrt(hx ** 2 + hy ** 2 + 1e-16)
    num = 2.0 * mx * my - alpha * mx * my + t                  # similarity_map, gmsd.jl:5-10
    den = mx ** 2 + my ** 2 - alpha * mx * my + t
    gms = num / den
    mean = gms.mean(axis=(0, 1, 2), keepdims=True)
    score = ((gms - mean) ** 2).mean(axis=(0, 1, 2))
    per = np.sqrt(score)
    return per.mean(), per


def peak_snr(x, y, peak_val=1.0):
    """psnr.jl:5-10 (the `mse == 0` branch compares an array with a scalar: never taken)."""
    mse = ((np.asarray(y, np.float64) - np.asarray(x, np.float64)) ** 2).mean(axis=(0, 1, 2))
    return np.mean(20.0 * np.log10(peak_val / np.sqrt(mse)))
