"""Image-quality losses and metrics of the training step -- host-side mirror of the reference's
src/metrics/ (gmsd.jl, ssim.jl, psnr.jl) over the HIP kernels in csrc/metrics_capi.hip.

Tensors are float32 (B, C, N, M) on a ROCm device (= Julia (M, N, C, B)); statistics are per image
over (M, N, C) as in the reference.  `gmsd` / `ssim` are differentiable w.r.t. their FIRST argument
(the model output in `loss_f(m(x), y)`, src/train.jl:52); the target gets no gradient.
There is no CPU path (host tensors raise TypeError)."""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .ops import Workspace

__all__ = ["gmsd", "gmsd_loss", "ssim", "ssim_loss", "ssim_loss_fast", "ssim_kernel", "peak_snr", "mse"]

# Gaussian, sigma 1.5, length 11 (ssim.jl:6-17)
SSIM_KERNEL = (0.00102838008447911, 0.007598758135239185, 0.03600077212843083, 0.10936068950970002,
               0.2130055377112537, 0.26601172486179436, 0.2130055377112537, 0.10936068950970002,
               0.03600077212843083, 0.007598758135239185, 0.00102838008447911)

_ws = {}


def _prep(x, y):
    for t in (x, y):
        if not isinstance(t, torch.Tensor) or t.device.type != "cuda" or t.dtype != torch.float32:
            raise TypeError("metrics: x and y must be float32 tensors on a ROCm device (no CPU path)")
    if x.shape != y.shape:
        raise ValueError(f"loss function expects size(ŷ) = {tuple(y.shape)} but is size {tuple(x.shape)}")   # ssim.jl:48
    if x.dim() < 2 or x.dim() > 4:
        raise ValueError("x must be 2-D .. 4-D (N, M) / (C, N, M) / (B, C, N, M)")
    x4 = x.reshape((1,) * (4 - x.dim()) + tuple(x.shape)).contiguous()
    return x4, y.reshape(x4.shape).contiguous()


def _workspace(dev, nbytes):
    """Scratch of a metrics call, one per (device, stream) as the solver's default workspaces
    (ops.Workspace): two losses enqueued on different streams never share scratch, and a growing
    reallocation is stream-ordered (the buffer is marked as used on the stream it serves)."""
    stream = torch.cuda.current_stream(dev)
    ws = _ws.setdefault((dev, stream.cuda_stream), Workspace())
    return ws.get(nbytes, dev, stream)


def _ws_for(x4, ks, grad):
    B, C, N, M = x4.shape
    out = ctypes.c_size_t(0)
    _lib.check(_lib.load().admm_metrics_workspace_bytes(M, N, C, B, ks, int(grad), ctypes.byref(out)))
    return _workspace(x4.device, out.value)


def _stream(dev):
    return torch.cuda.current_stream(dev).cuda_stream


def _gmsd_call(x4, y4, t, alpha, out_bar=None, want_grad=False):
    B, C, N, M = x4.shape
    per = torch.empty(B, dtype=torch.float32, device=x4.device)
    xb = torch.empty_like(x4) if want_grad else None
    wp, wl = _ws_for(x4, 0, want_grad)
    ob = out_bar.contiguous().to(torch.float32) if out_bar is not None else None
    _lib.check(_lib.load().admm_gmsd_f32(x4.data_ptr(), y4.data_ptr(), M, N, C, B, float(t), float(alpha),
                                         per.data_ptr(), None if ob is None else ob.data_ptr(),
                                         None if xb is None else xb.data_ptr(), wp, wl, _stream(x4.device)))
    return per, xb


class _GmsdFn(torch.autograd.Function):
    """The forward keeps its own workspace when x needs a gradient: it holds the per-block partial sums, from which
    admm_gmsd_backward_f32 forms the gradient without re-running the forward kernel."""

    @staticmethod
    def forward(ctx, x4, y4, t, alpha):
        ctx.save_for_backward(x4, y4)
        ctx.t, ctx.alpha = t, alpha
        if not ctx.needs_input_grad[0]:
            return _gmsd_call(x4, y4, t, alpha)[0]
        B, C, N, M = x4.shape
        nb = ctypes.c_size_t(0)
        _lib.check(_lib.load().admm_metrics_workspace_bytes(M, N, C, B, 0, 1, ctypes.byref(nb)))
        ctx.ws = Workspace()   # private: a second loss before backward must not overwrite these sums
        wp, wl = ctx.ws.get(nb.value, x4.device, torch.cuda.current_stream(x4.device))
        per = torch.empty(B, dtype=torch.float32, device=x4.device)
        _lib.check(_lib.load().admm_gmsd_f32(x4.data_ptr(), y4.data_ptr(), M, N, C, B, float(t), float(alpha),
                                             per.data_ptr(), None, None, wp, wl, _stream(x4.device)))
        return per

    @staticmethod
    def backward(ctx, gper):
        x4, y4 = ctx.saved_tensors
        B, C, N, M = x4.shape
        xb = torch.empty_like(x4)
        ob = gper.contiguous().to(torch.float32)
        wp, wl = ctx.ws.get(0, x4.device, torch.cuda.current_stream(x4.device))
        _lib.check(_lib.load().admm_gmsd_backward_f32(x4.data_ptr(), y4.data_ptr(), M, N, C, B, float(ctx.t),
                                                      float(ctx.alpha), ob.data_ptr(), xb.data_ptr(), wp, wl,
                                                      _stream(x4.device)))
        ctx.ws = None
        return xb, None, None, None


def gmsd(x, y, t=0.0026, alpha=0.0, reduction=torch.mean):
    """gmsd(x, y, t=0.0026f0, α=0f0, reduction=Flux.mean) -- gmsd.jl:13-27: per-image gradient
    magnitude similarity deviation (Sobel gradients on the circular padding), reduced over the batch."""
    x4, y4 = _prep(x, y)
    per = _GmsdFn.apply(x4, y4, float(t), float(alpha))
    return reduction(per)


gmsd_loss = gmsd   # gmsd.jl:29


def ssim_kernel(kernel_length=None):
    """1-D taps of the separable SSIM window: the Gaussian (σ 1.5, length 11) of ssim.jl:23, or the
    normalised box of ssim_loss_fast (ssim.jl:160) when kernel_length is given."""
    if kernel_length is None:
        return SSIM_KERNEL
    return (1.0 / kernel_length,) * int(kernel_length)


def _taps(kernel):
    if kernel is None:
        return SSIM_KERNEL
    if isinstance(kernel, torch.Tensor):
        k = kernel.detach().to("cpu", torch.float64)
        if k.dim() >= 2:   # a separable 2-D (or (k, k, 1, C)) kernel: recover the 1-D factor
            k2 = k.reshape(k.shape[0], k.shape[1], -1)[:, :, 0] if k.dim() > 2 else k
            col = k2.sum(dim=1)
            row = k2.sum(dim=0)
            if not torch.allclose(torch.outer(col, row) / k2.sum(), k2, atol=1e-7):
                raise ValueError("ssim: only separable windows are supported")
            if not torch.allclose(col, row):
                raise ValueError("ssim: the window must be the same along both dims")
            k = col / col.sum().sqrt() * (k2.sum().sqrt() / col.sum().sqrt())
        return tuple(float(v) for v in k.reshape(-1))
    return tuple(float(v) for v in kernel)


def _ssim_call(x4, y4, taps, peak, crop, out_bar=None, want_grad=False):
    B, C, N, M = x4.shape
    ks = len(taps)
    per = torch.empty(B, dtype=torch.float32, device=x4.device)
    xb = torch.empty_like(x4) if want_grad else None
    wp, wl = _ws_for(x4, ks, want_grad)
    tk = (ctypes.c_float * ks)(*taps)
    ob = out_bar.contiguous().to(torch.float32) if out_bar is not None else None
    _lib.check(_lib.load().admm_ssim_f32(x4.data_ptr(), y4.data_ptr(), M, N, C, B, tk, ks, float(peak), int(bool(crop)),
                                         per.data_ptr(), None if ob is None else ob.data_ptr(),
                                         None if xb is None else xb.data_ptr(), wp, wl, _stream(x4.device)))
    return per, xb


class _SsimFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x4, y4, taps, peak, crop):
        ctx.save_for_backward(x4, y4)
        ctx.taps, ctx.peak, ctx.crop = taps, peak, crop
        return _ssim_call(x4, y4, taps, peak, crop)[0]

    @staticmethod
    def backward(ctx, gper):
        x4, y4 = ctx.saved_tensors
        _, xb = _ssim_call(x4, y4, ctx.taps, ctx.peak, ctx.crop, out_bar=gper, want_grad=True)
        return xb, None, None, None, None


def ssim(x, y, kernel=None, *, peakval=1.0, crop=True, dims=None):
    """ssim(x, y, kernel=ssim_kernel(x); peakval=1, crop=true) -- ssim.jl:84-124: mean over images of
    the mean SSIM map (valid window when crop, else same-size on the symmetric padding).  `dims` is
    accepted and, as in the reference, not used."""
    x4, y4 = _prep(x, y)
    per = _SsimFn.apply(x4, y4, _taps(kernel), float(peakval), bool(crop))
    return per.mean()


def ssim_loss(x, y, kernel=None, **kw):
    """1 - ssim(x, y) (ssim.jl:148)."""
    return 1.0 - ssim(x, y, kernel, **kw)


def ssim_loss_fast(x, y, kernel_length=5, **kw):
    """ssim_loss with a normalised kernel_length^2 box window (ssim.jl:160-164)."""
    return ssim_loss(x, y, ssim_kernel(kernel_length), **kw)


def _mse_per_image(x4, y4):
    B, C, N, M = x4.shape
    per = torch.empty(B, dtype=torch.float32, device=x4.device)
    wp, wl = _ws_for(x4, 0, False)
    _lib.check(_lib.load().admm_mse_f32(x4.data_ptr(), y4.data_ptr(), M, N, C, B, per.data_ptr(), wp, wl,
                                        _stream(x4.device)))
    return per


def peak_snr(x, y, peak_val=1.0):
    """peak_snr(x, y, peak_val=1f0) -- psnr.jl:5-10: mean over images of 20 log10(peak / sqrt(mse)).
    (The reference's `mse == 0` guard compares an array with a scalar and never fires; kept as is.)"""
    x4, y4 = _prep(x, y)
    per = _mse_per_image(x4.detach(), y4.detach())
    return torch.mean(20.0 * torch.log10(peak_val / torch.sqrt(per)))


def mse(x, y):
    """Flux.mse(x, y) = mean((x - y)^2) over every element (src/train.jl:131), via the per-image kernel."""
    x4, y4 = _prep(x, y)
    return _mse_per_image(x4.detach(), y4.detach()).mean()
