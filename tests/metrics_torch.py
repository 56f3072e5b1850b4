"""fp64 PyTorch restatement of the metrics (same formulas as oracle/oracle_metrics.py) for the
GRADIENT checks of the HIP kernels: torch autograd differentiates it.  Tensors (B, C, N, M)."""
import torch
import torch.nn.functional as F

import oracle_metrics as om


def _dwconv(x, K):
    """NNlib conv (flipped kernel), per channel, valid; K indexed [a (dim 1 = M), b (dim 2 = N)]."""
    B, C, N, M = x.shape
    w = torch.as_tensor(K[::-1, ::-1].T.copy(), dtype=x.dtype)      # torch weight [kN][kM]
    w = w.reshape(1, 1, *w.shape).repeat(C, 1, 1, 1)
    return F.conv2d(x, w, groups=C)                                  # cross-correlation with the flip


def ssim_per_image(x, y, kernel=None, peakval=1.0):
    k = om.SSIM_KERNEL if kernel is None else kernel
    import numpy as np
    K = np.outer(k, k)
    C1, C2 = (peakval * 0.01) ** 2, (peakval * 0.03) ** 2
    mx, my = _dwconv(x, K), _dwconv(y, K)
    sx = _dwconv(x * x, K) - mx * mx
    sy = _dwconv(y * y, K) - my * my
    sxy = _dwconv(x * y, K) - mx * my
    s = (2 * mx * my + C1) * (2 * sxy + C2) / ((mx * mx + my * my + C1) * (sx + sy + C2))
    return s.mean(dim=(1, 2, 3))


def gmsd_per_image(x, y, t=0.0026, alpha=0.0):
    def grads(z):
        zp = F.pad(z, (1, 1, 1, 1), mode="circular")
        return _dwconv(zp, om.SOBEL_KERNEL_X), _dwconv(zp, om.SOBEL_KERNEL_Y)
    gx, gy = grads(x)
    hx, hy = grads(y)
    mx = torch.sqrt(gx ** 2 + gy ** 2 + 1e-16)
    my = torch.sqrt(hx ** 2 + hy ** 2 + 1e-16)
    g = (2 * mx * my - alpha * mx * my + t) / (mx ** 2 + my ** 2 - alpha * mx * my + t)
    mean = g.mean(dim=(1, 2, 3), keepdim=True)
    return torch.sqrt(((g - mean) ** 2).mean(dim=(1, 2, 3)))
