"""`tvd_fft` -- host-side mirror of the reference operator
`tvd_fft(y, λ, ρ, h, isotropic=false, maxit=100)` (/root/reference/src/ops/ops.jl:181-188).

The reference dispatches on the array type (`typeof(y) <: CuArray` -> tvd_fft_gpu, ops.jl:183);
here the device array is a torch tensor on a ROCm device and the body is the HIP library behind
the C ABI (include/admm_deconv.h).  Host (CPU) tensors are rejected: this package has no CPU
path (the CPU restatement under oracle/ is test infrastructure only).

Layout: a torch tensor of shape (B, P, N, M), C-contiguous float32, is byte-identical to the
reference's Julia array (M, N, P, B).  The PSF h is torch (kw, kh) == Julia (kh, kw).
"""
from __future__ import annotations

import math

import torch

from . import _lib

__all__ = ["tvd_fft", "Workspace"]


class Workspace:
    """Caller-owned device scratch for the solve (the library allocates nothing)."""

    def __init__(self):
        self._buf = None

    def get(self, nbytes, device):
        if self._buf is None or self._buf.numel() < nbytes or self._buf.device != device:
            self._buf = torch.empty(max(nbytes, 256) + 256, dtype=torch.uint8, device=device)
        ptr = self._buf.data_ptr()
        off = (-ptr) % 256
        return ptr + off, self._buf.numel() - off


_default_ws = {}


def _scalar(v, name):
    if isinstance(v, torch.Tensor):
        if v.numel() != 1:
            raise ValueError(f"{name} must have exactly one element (reference uses 1-element vectors)")
        v = v.detach().reshape(-1)[0].item()
    elif hasattr(v, "__len__"):
        if len(v) != 1:
            raise ValueError(f"{name} must have exactly one element")
        v = v[0]
    v = float(v)
    if not math.isfinite(v):
        raise ValueError(f"{name} must be finite")
    return v


def tvd_fft(y, lam, rho=1.0, h=None, isotropic=False, maxit=100, *, out=None, workspace=None, stream=None):
    """ADMM TV deconvolution of every (M x N) plane of y (ops.jl:181).

    y:    torch float32 tensor (B, P, N, M) on a ROCm device (Julia (M,N,P,B)); a 2-D (N, M) or
          3-D (P, N, M) tensor is treated as B = 1 (and P = 1).
    lam, rho: scalars or 1-element tensors (the reference's 1-element vectors; default ρ = [1]).
    h:    PSF tensor (kw, kh) (Julia (kh,kw,1,1)), or None / empty for the reference's empty PSF.
    Returns a new tensor x of y's shape (y is not modified)."""
    if not isinstance(y, torch.Tensor) or y.device.type != "cuda":
        raise TypeError("tvd_fft: y must be a torch tensor on a ROCm device (no CPU path in this package)")
    if y.dtype != torch.float32:
        raise TypeError("tvd_fft: y must be float32 (the reference's T)")
    shape = y.shape
    if y.dim() == 2:
        y4 = y.reshape(1, 1, *shape)
    elif y.dim() == 3:
        y4 = y.reshape(1, *shape)
    elif y.dim() == 4:
        y4 = y
    else:
        raise ValueError("tvd_fft: y must be 2-D, 3-D or 4-D")
    y4 = y4.contiguous()
    B, P, N, M = y4.shape
    lam = _scalar(lam, "lambda")
    rho = _scalar(rho, "rho")
    if h is None or (isinstance(h, torch.Tensor) and h.numel() == 0):
        hp, kh, kw, hbuf = None, 0, 0, None
    else:
        hbuf = h.detach()
        while hbuf.dim() > 2 and hbuf.shape[0] == 1:
            hbuf = hbuf[0]
        if hbuf.dim() != 2:
            raise ValueError("PSF must be 2-D (kw, kh)")
        hbuf = hbuf.to(device=y.device, dtype=torch.float32).contiguous()
        kw, kh = hbuf.shape
        hp = hbuf.data_ptr()
    if out is None:
        out = torch.empty_like(y4)
    elif out.shape != y4.shape or out.dtype != torch.float32 or not out.is_contiguous() or out.device != y.device:
        raise ValueError("out must be a contiguous float32 tensor of y's shape on y's device")
    nbytes = _lib.workspace_bytes(M, N, P, B, kh, kw, isotropic)
    if workspace is None:
        workspace = _default_ws.setdefault(y.device, Workspace())
    ws_ptr, ws_len = workspace.get(nbytes, y.device)
    if stream is None:
        stream = torch.cuda.current_stream(y.device)
    s_handle = stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)
    _lib.check(_lib.load().admm_tvd_forward_f32(
        y4.data_ptr(), out.data_ptr(), M, N, P, B, hp, kh, kw, lam, rho, int(bool(isotropic)), int(maxit),
        ws_ptr, ws_len, s_handle))
    return out.reshape(shape)
