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

import contextlib
import ctypes
import math

import torch

from . import _lib

__all__ = ["tvd_fft", "tvd_fft_backward", "tvd_fft_record", "tvd_fft_backward_recorded", "Recording", "Workspace",
           "tvd_fft_multi", "tvd_fft_multi_backward_recorded", "multi_supported"]


class Workspace:
    """Caller-owned device scratch for the solve (the library allocates nothing).

    A workspace serves one stream at a time: the solve's scratch state (C table, H^T y, s, spectra)
    lives in it for the whole enqueued solve.  `get(nbytes, device, stream)` marks the buffer as used on
    `stream`, so that a reallocation (or dropping the workspace) does not hand the memory to other work
    before that stream has finished with it."""

    def __init__(self):
        self._buf = None

    def get(self, nbytes, device, stream=None):
        # + 256: room for the 256-B alignment of the returned pointer
        if self._buf is None or self._buf.numel() < nbytes + 256 or self._buf.device != device:
            self._buf = torch.empty(max(nbytes, 256) + 256, dtype=torch.uint8, device=device)
        if stream is not None and isinstance(stream, torch.cuda.Stream) and stream != torch.cuda.current_stream(device):
            self._buf.record_stream(stream)
        ptr = self._buf.data_ptr()
        off = (-ptr) % 256
        return ptr + off, self._buf.numel() - off


# default workspaces, one per (kind, device, stream): concurrent solves on different streams (e.g. the
# branches of layers.Parallel) must not share scratch state
_default_ws = {}


def _default_workspace(kind, device, stream):
    return _default_ws.setdefault((kind, device, _stream_handle(stream)), Workspace())


def _stream_handle(stream):
    return stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)


def _make_reducer(workspace, group):
    """admm_batch_reducer for a batch sharded over `group` (isotropic prox; include/admm_deconv.h).

    The library hands over a device pointer into `workspace` holding this shard's M x N partial map;
    the callback all-reduces (sum) that slice of the workspace tensor in place, on the library's
    stream.  gloo (CPU-only collectives) goes through a host copy.  Returns (struct, keep-alive)."""
    import torch.distributed as dist

    def cb(buf, count, stream, _user):
        try:
            base = workspace._buf.data_ptr()
            off = int(buf) - base
            view = workspace._buf[off: off + 4 * int(count)].view(torch.float32)
            ctx, lib_stream = contextlib.nullcontext(), None
            if view.is_cuda:
                # the stream the library enqueued the map on: handle 0 is torch's own default stream object (an
                # ExternalStream wrapped around handle 0 did not order torch's copies after the library's kernels:
                # a second sharded call read the map early, tests/test_gpu_dist_iso.py, round 6)
                h = int(stream or 0)
                cur = torch.cuda.current_stream(view.device)
                lib_stream = (cur if cur.cuda_stream == h else torch.cuda.default_stream(view.device) if h == 0
                              else torch.cuda.ExternalStream(h, device=view.device))
                ctx = torch.cuda.stream(lib_stream)
            with ctx:
                if dist.get_backend(group) == "gloo":
                    # host round trip (test infrastructure: gloo carries CPU tensors); the library launches its next
                    # kernel as soon as this returns, so the copy back must have landed by then
                    host = view.cpu()
                    dist.all_reduce(host, group=group)
                    view.copy_(host)
                    if lib_stream is not None:
                        lib_stream.synchronize()
                else:
                    dist.all_reduce(view, group=group)   # enqueued behind the library's work on its stream
            return 0
        except BaseException as e:   # an exception must not unwind through the C frames
            import sys
            print(f"admm_deconv batch reducer failed: {e!r}", file=sys.stderr)
            return -1

    fn = _lib.REDUCE_FN(cb)
    return _lib.BatchReducer(fn, None), fn


def _sharded(isotropic, group):
    if group is None or not isotropic:
        return False
    import torch.distributed as dist
    return dist.is_initialized() and dist.get_world_size(group) > 1


class _DevScalars:
    """lambda / rho as device fp32 1-element tensors (the reference's `λ::CGPUArray`, ops.jl:99,181): the
    library reads them in-kernel, so the call needs no device-to-host read.  Holds the (possibly
    converted) tensors alive; `ptrs` are their device addresses."""

    __slots__ = ("lam", "rho")

    def __init__(self, lam, rho, device, stream):
        self.lam = self._one(lam, "lambda", device)
        self.rho = self._one(rho, "rho", device)
        if stream is not None and isinstance(stream, torch.cuda.Stream) and stream != torch.cuda.current_stream(device):
            for t in (self.lam, self.rho):
                t.record_stream(stream)

    @staticmethod
    def _one(v, name, device):
        if isinstance(v, torch.Tensor):
            if v.numel() != 1:
                raise ValueError(f"{name} must have exactly one element (reference uses 1-element vectors)")
            t = v.detach().reshape(1)
            if t.device != device:
                if t.device.type == "cuda":
                    raise ValueError(f"{name} is on {t.device}, the solve on {device}")
                t = t.to(device)            # host tensor: one (blocking) upload
            return t.to(torch.float32).contiguous()
        # a host number next to a device tensor: a fill on the device, no transfer
        return torch.full((1,), _scalar(v, name), dtype=torch.float32, device=device)

    @property
    def ptrs(self):
        return self.lam.data_ptr(), self.rho.data_ptr()


def _on_device(lam, rho):
    return any(isinstance(v, torch.Tensor) and v.device.type == "cuda" for v in (lam, rho))


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


def _stream_of(stream, device):
    if stream is None:
        stream = torch.cuda.current_stream(device)
    return stream, _stream_handle(stream)


def _forward_raw(y, lam, rho=1.0, h=None, isotropic=False, maxit=100, *, out=None, workspace=None, stream=None,
                 group=None):
    """ADMM TV deconvolution of every (M x N) plane of y (ops.jl:181).

    y:    torch float32 tensor (B, P, N, M) on a ROCm device (Julia (M,N,P,B)); a 2-D (N, M) or
          3-D (P, N, M) tensor is treated as B = 1 (and P = 1).
    lam, rho: host scalars, or 1-element tensors (the reference's 1-element vectors; default ρ = [1]).
          Device tensors are read in-kernel (admm_tvd_forward_dev_f32): no host synchronisation.
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
    stream, s_handle = _stream_of(stream, y.device)
    nbytes = _lib.workspace_bytes(M, N, P, B, kh, kw, isotropic)
    if workspace is None:
        workspace = _default_workspace("fwd", y.device, stream)
    ws_ptr, ws_len = workspace.get(nbytes, y.device, stream)
    red, keep = _make_reducer(workspace, group) if _sharded(isotropic, group) else (None, None)
    if _on_device(lam, rho):
        dv = _DevScalars(lam, rho, y.device, stream)
        _lib.check(_lib.load().admm_tvd_forward_dev_f32(
            y4.data_ptr(), out.data_ptr(), M, N, P, B, hp, kh, kw, *dv.ptrs, int(bool(isotropic)), int(maxit),
            ws_ptr, ws_len, s_handle, ctypes.byref(red) if red is not None else None))
    elif red is not None:
        _lib.check(_lib.load().admm_tvd_forward_sharded_f32(
            y4.data_ptr(), out.data_ptr(), M, N, P, B, hp, kh, kw, _scalar(lam, "lambda"), _scalar(rho, "rho"), 1,
            int(maxit), ws_ptr, ws_len, s_handle, ctypes.byref(red)))
    else:
        _lib.check(_lib.load().admm_tvd_forward_f32(
            y4.data_ptr(), out.data_ptr(), M, N, P, B, hp, kh, kw, _scalar(lam, "lambda"), _scalar(rho, "rho"),
            int(bool(isotropic)), int(maxit), ws_ptr, ws_len, s_handle))
    del keep
    return out.reshape(shape)


def _prep(y, h):
    if not isinstance(y, torch.Tensor) or y.device.type != "cuda" or y.dtype != torch.float32:
        raise TypeError("y must be a float32 torch tensor on a ROCm device (no CPU path in this package)")
    shape = y.shape
    y4 = y.reshape((1,) * (4 - y.dim()) + tuple(shape)).contiguous() if y.dim() < 4 else y.contiguous()
    if h is None or h.numel() == 0:
        return shape, y4, None
    hb = h.detach()
    while hb.dim() > 2 and hb.shape[0] == 1:
        hb = hb[0]
    return shape, y4, hb.to(device=y.device, dtype=torch.float32).contiguous()


def _scalars_for(lam, rho, device, stream):
    """(device holder or None, host lambda, host rho): device tensors stay on the device."""
    if _on_device(lam, rho):
        return _DevScalars(lam, rho, device, stream), None, None
    return None, _scalar(lam, "lambda"), _scalar(rho, "rho")


def tvd_fft_backward(y, x_bar, lam, rho=1.0, h=None, isotropic=False, maxit=100, *, need_h=True, need_y=True,
                     need_rho=True, workspace=None, stream=None, group=None):
    """Adjoint of tvd_fft through all `maxit` unrolled iterations (what Zygote computes for the
    reference, src/train.jl:51).  Returns (x, y_bar, h_bar, lam_bar, rho_bar); h_bar is None without a PSF
    or when need_h is False; y_bar is None when need_y is False (the sweep then keeps no running sum of
    vbar unless h_bar needs it: 8 B/px less traffic per reverse step); rho_bar is None when need_rho is
    False (the fused and isotropic sweeps then skip s_k, which only rho_bar reads).  Recomputes the forward
    (x is returned for convenience).
    With `group` (isotropic prox, batch sharded over the group's ranks) h_bar / lam_bar / rho_bar are
    this shard's contributions: their sum over ranks is the gradient of the whole batch."""
    shape, y4, hb = _prep(y, h)
    B, P, N, M = y4.shape
    xb = x_bar.reshape(y4.shape).to(torch.float32).contiguous()
    kw, kh = (0, 0) if hb is None else hb.shape
    want_h = need_h and hb is not None
    stream, s_handle = _stream_of(stream, y.device)
    dv, lam_h, rho_h = _scalars_for(lam, rho, y.device, stream)
    nbytes = _lib.backward_workspace_bytes(M, N, P, B, kh, kw, isotropic, maxit, want_h)
    if workspace is None:
        workspace = _default_workspace("bwd", y.device, stream)
    ws_ptr, ws_len = workspace.get(nbytes, y.device, stream)
    x = torch.empty_like(y4)
    y_bar = torch.empty_like(y4) if need_y else None
    h_bar = torch.empty_like(hb) if want_h else None
    scal = torch.zeros(2, dtype=torch.float32, device=y.device)
    head = (y4.data_ptr(), xb.data_ptr(), y_bar.data_ptr() if need_y else None, h_bar.data_ptr() if want_h else None, scal.data_ptr(),
            scal.data_ptr() + 4 if need_rho else None, M, N, P, B, None if hb is None else hb.data_ptr(), kh, kw)
    tail = (int(bool(isotropic)), int(maxit), x.data_ptr(), ws_ptr, ws_len, s_handle)
    red, keep = _make_reducer(workspace, group) if _sharded(isotropic, group) else (None, None)
    L = _lib.load()
    if dv is not None:
        _lib.check(L.admm_tvd_backward_dev_f32(*head, *dv.ptrs, *tail, ctypes.byref(red) if red is not None else None))
    elif red is not None:
        _lib.check(L.admm_tvd_backward_sharded_f32(*head, lam_h, rho_h, *tail, ctypes.byref(red)))
    else:
        _lib.check(L.admm_tvd_backward_f32(*head, lam_h, rho_h, *tail))
    del keep
    return x.reshape(shape), y_bar.reshape(shape) if need_y else None, h_bar, scal[0], scal[1] if need_rho else None


class Recording:
    """One forward solve recorded for its adjoint (admm_tvd_forward_record_f32): the trajectory lives in
    its own workspace until tvd_fft_backward_recorded consumes it, so a training step runs the forward
    once (no recompute in the backward).  Memory: about 8 B/px per iteration (plus 8 B/px of dim-2
    spectra per iteration with a PSF when h_bar is needed) -- sized for MI355X's 288 GB HBM."""

    __slots__ = ("workspace", "y4", "hb", "shape", "dv", "lam", "rho", "iso", "maxit", "want_h", "group", "dims",
                 "flags")


def tvd_fft_record(y, lam, rho=1.0, h=None, isotropic=False, maxit=100, *, need_h=True, need_rho=True, stream=None,
                   group=None):
    """Forward solve that records its trajectory.  Returns (x, Recording); see tvd_fft_backward_recorded.
    lam / rho as device tensors are read in-kernel (no host sync), as in tvd_fft.  need_rho=False: the
    replay will not be asked for rho_bar, so the fused 256 x 256 anisotropic path records only the
    soft-threshold branch of every trajectory element (ADMM_REC_MASKS: 16x less memory, a cheaper reverse
    sweep, the other gradients bitwise the same)."""
    shape, y4, hb = _prep(y, h)
    B, P, N, M = y4.shape
    stream, s_handle = _stream_of(stream, y.device)
    rec = Recording()
    rec.dv, rec.lam, rec.rho = _scalars_for(lam, rho, y.device, stream)
    kw, kh = (0, 0) if hb is None else hb.shape
    rec.want_h = bool(need_h and hb is not None)
    rec.y4, rec.hb, rec.shape, rec.iso, rec.maxit, rec.group = y4, hb, shape, bool(isotropic), int(maxit), group
    rec.dims = (M, N, P, B, kh, kw)
    rec.flags = (_lib.REC_HBAR if rec.want_h else 0) | (0 if need_rho else _lib.REC_MASKS)
    nbytes = _lib.backward_workspace_bytes(M, N, P, B, kh, kw, isotropic, maxit, rec.flags)
    rec.workspace = Workspace()
    ws_ptr, ws_len = rec.workspace.get(nbytes, y.device, stream)
    x = torch.empty_like(y4)
    red, keep = _make_reducer(rec.workspace, group) if _sharded(isotropic, group) else (None, None)
    head = (y4.data_ptr(), x.data_ptr(), M, N, P, B, None if hb is None else hb.data_ptr(), kh, kw)
    tail = (int(rec.iso), rec.maxit, rec.flags, ws_ptr, ws_len, s_handle,
            ctypes.byref(red) if red is not None else None)
    L = _lib.load()
    if rec.dv is not None:
        _lib.check(L.admm_tvd_forward_record_dev_f32(*head, *rec.dv.ptrs, *tail))
    else:
        _lib.check(L.admm_tvd_forward_record_f32(*head, rec.lam, rec.rho, *tail))
    del keep
    return x.reshape(shape), rec


def tvd_fft_backward_recorded(rec, x, x_bar, *, stream=None, need_y=True, need_rho=True):
    """Reverse sweep of a recorded forward (x = that forward's output, unmodified).  Returns
    (y_bar, h_bar, lam_bar, rho_bar); h_bar is None unless the forward was recorded with need_h, y_bar is
    None when need_y is False (cheaper: no running sum of vbar unless h_bar needs it), rho_bar is None when
    need_rho is False (cheaper: the fused and isotropic sweeps then skip s_k, read for rho_bar only).
    Consumes the recording (its workspace is released)."""
    if rec.workspace is None:
        raise RuntimeError("recording already consumed")
    M, N, P, B, kh, kw = rec.dims
    y4, hb = rec.y4, rec.hb
    xb = x_bar.reshape(y4.shape).to(torch.float32).contiguous()
    x4 = x.reshape(y4.shape)
    if not x4.is_contiguous():
        raise ValueError("x must be the recorded forward's (contiguous) output")
    stream, s_handle = _stream_of(stream, y4.device)
    ws = rec.workspace
    ws_ptr, ws_len = ws.get(0, y4.device, stream)
    y_bar = torch.empty_like(y4) if need_y else None
    h_bar = torch.empty_like(hb) if rec.want_h else None
    scal = torch.zeros(2, dtype=torch.float32, device=y4.device)
    red, keep = _make_reducer(ws, rec.group) if _sharded(rec.iso, rec.group) else (None, None)
    head = (y4.data_ptr(), xb.data_ptr(), y_bar.data_ptr() if need_y else None, h_bar.data_ptr() if rec.want_h else None, scal.data_ptr(),
            scal.data_ptr() + 4 if need_rho else None, M, N, P, B, None if hb is None else hb.data_ptr(), kh, kw)
    tail = (int(rec.iso), rec.maxit, x4.data_ptr(), ws_ptr, ws_len, s_handle,
            ctypes.byref(red) if red is not None else None)
    L = _lib.load()
    if rec.dv is not None:
        if isinstance(stream, torch.cuda.Stream) and stream != torch.cuda.current_stream(y4.device):
            for t in (rec.dv.lam, rec.dv.rho):
                t.record_stream(stream)
        _lib.check(L.admm_tvd_backward_recorded_dev_f32(*head, *rec.dv.ptrs, *tail))
    else:
        _lib.check(L.admm_tvd_backward_recorded_f32(*head, rec.lam, rec.rho, *tail))
    del keep
    rec.workspace = None    # released once the stream has consumed it (caching allocator is stream-ordered)
    return y_bar.reshape(rec.shape) if need_y else None, h_bar, scal[0], scal[1] if need_rho else None


class _TvdFFTFn(torch.autograd.Function):
    """Differentiable tvd_fft: forward through the HIP solve, backward through the HIP adjoint
    (the rrule the Julia shim would register, julia/ADMMDeconvHIP.jl)."""

    @staticmethod
    def forward(ctx, y, lam_t, rho_t, h_t, isotropic, maxit, group, scalars):
        # the forward records its trajectory; the backward runs only the reverse sweep from it.  lam_t / rho_t
        # (device tensors) are read in-kernel unless the caller handed their host values in `scalars`
        need_h = h_t.numel() > 0 and ctx.needs_input_grad[3]
        lam, rho = scalars if scalars is not None else (lam_t, rho_t)
        # rho not trainable here (ADMMDeconvF2, F3): the recording keeps only the ST branches when it can
        x, ctx.rec = tvd_fft_record(y, lam, rho, h_t if h_t.numel() else None, isotropic, maxit,
                                    need_h=need_h, need_rho=ctx.needs_input_grad[2], group=group)
        # y (read again by the reverse sweep's h_bar correlation) and x are version-checked: an in-place
        # change of either between forward and backward raises instead of giving a wrong gradient
        ctx.save_for_backward(y, lam_t, rho_t, h_t, x)
        return x

    @staticmethod
    def backward(ctx, x_bar):
        _y, lam_t, rho_t, h_t, x = ctx.saved_tensors
        need_h = ctx.rec.want_h
        # y_bar only when y needs it (a first-layer denoiser's input does not): the sweep then skips Vsum
        yb, hb, lb, rb = tvd_fft_backward_recorded(ctx.rec, x, x_bar, need_y=ctx.needs_input_grad[0],
                                                   need_rho=ctx.needs_input_grad[2])
        ctx.rec = None
        hg = None
        if need_h:
            hg = hb.reshape(h_t.shape)
        return (yb if ctx.needs_input_grad[0] else None,
                lb.reshape(lam_t.shape).to(lam_t.dtype) if ctx.needs_input_grad[1] else None,
                rb.reshape(rho_t.shape).to(rho_t.dtype) if ctx.needs_input_grad[2] else None,
                hg, None, None, None, None)


def tvd_fft(y, lam, rho=1.0, h=None, isotropic=False, maxit=100, *, out=None, workspace=None, stream=None,
            group=None, scalars=None):
    """ADMM TV deconvolution of every (M x N) plane of y -- src/ops/ops.jl:181 semantics.

    y: float32 tensor (B,P,N,M) on a ROCm device (= Julia (M,N,P,B)); lam, rho: host scalars or
    1-element tensors -- device tensors (the reference's `λ::CGPUArray`) are read in-kernel, so the call
    never synchronises the host; h: PSF (kw,kh) (= Julia (kh,kw)) or None/empty.  Returns a new tensor.
    Differentiable (y, lam, rho, h) when autograd is recording and any of them requires grad
    (either prox); the gradient is the exact adjoint of the K unrolled iterations.
    group: torch.distributed group the batch is sharded over (each rank passes its own slice).  The
    isotropic prox's pixelnorm then spans the whole sharded batch (one M x N all-reduce per
    iteration), so every rank gets its slice of the unsharded result; ignored for the anisotropic
    prox, whose planes are independent.
    scalars: optional host (lambda, rho) equal to the values of tensor lam / rho, used instead of the
    device values (gradients still flow to the tensors)."""
    tensors = [t for t in (y, lam, rho, h) if isinstance(t, torch.Tensor)]
    if torch.is_grad_enabled() and any(t.requires_grad for t in tensors):
        dev = y.device
        as_t = lambda v: v if isinstance(v, torch.Tensor) else torch.full((1,), float(v), device=dev)  # noqa: E731
        h_t = h if isinstance(h, torch.Tensor) else torch.zeros(0, device=dev)
        return _TvdFFTFn.apply(y, as_t(lam), as_t(rho), h_t, bool(isotropic), int(maxit), group, scalars)
    if scalars is not None:
        lam, rho = scalars
    return _forward_raw(y, lam, rho, h, isotropic, maxit, out=out, workspace=workspace, stream=stream, group=group)


# ---- several ADMM branches of one shared input (Parallel(chcat, ...), src/nets/net_build.jl:113-125) ----
MULTI_M = MULTI_N = 256


def multi_supported(y, isotropic=False, psf=None, group=None):
    """Whether the one-grid multi-branch solve (admm_tvd_forward_multi_dev_f32) covers this input: the fused
    256 x 256 kernels (anisotropic, or isotropic with the fused reverse sweep on), no PSF, one process
    holding the batch, and the fused option on."""
    return (isinstance(y, torch.Tensor) and y.is_cuda and y.dtype == torch.float32 and y.dim() == 4
            and y.shape[-1] == MULTI_M and y.shape[-2] == MULTI_N
            and (not isotropic or _lib.get_option("FUSED_ADJ") == 1)
            and (psf is None or psf.numel() == 0) and group is None and _lib.get_option("FUSED") == 1)


class MultiRecording:
    """A multi-branch forward recorded for its reverse sweep (tvd_fft_multi(record=True))."""
    __slots__ = ("workspace", "dims", "maxit", "masks", "dv")


def _ptr_array(ts):
    return (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])


def tvd_fft_multi(y, lams, rhos, maxit=100, *, out=None, record=False, need_rho=True, isotropic=False, workspace=None,
                  stream=None):
    """x = chcat(tvd_fft(y, lams[0], rhos[0], nothing, false, maxit), ..., tvd_fft(y, lams[n-1], ...)) in ONE
    launch of the fused kernel (every branch's planes in one grid).  y: (B, P, 256, 256) float32 on the
    device; lams, rhos: n 1-element tensors / numbers (device tensors read in-kernel).  Returns x of shape
    (B, n * P, 256, 256) -- the chcat layout, branch i's channels at i*P..i*P+P-1 -- and, with record=True,
    a MultiRecording for tvd_fft_multi_backward_recorded (need_rho=False: only the ST branches are kept).
    isotropic=True: the BT prox (ops.jl:6,10), each branch's norm over its own planes; its recording never
    gives rho_bar (the fused isotropic sweep, plane_iso.hip)."""
    if not multi_supported(y, isotropic):
        raise ValueError("tvd_fft_multi: y must be a float32 (B, P, 256, 256) ROCm tensor (fused options on)")
    if record and isotropic and need_rho:
        raise ValueError("tvd_fft_multi: an isotropic recording gives lambda_bar and y_bar only (need_rho=False)")
    n = len(lams)
    if n < 1 or len(rhos) != n:
        raise ValueError("tvd_fft_multi: one lambda and one rho per branch")
    y4 = y.contiguous()
    B, P, N, M = y4.shape
    stream, s_handle = _stream_of(stream, y.device)
    dv = [_DevScalars(l, r, y.device, stream) for l, r in zip(lams, rhos)]
    flags = (_lib.MULTI_RECORD | (0 if need_rho else _lib.REC_MASKS)) if record else 0
    if isotropic:
        flags |= _lib.MULTI_ISO
    nbytes = _lib.multi_workspace_bytes(M, N, P, B, n, maxit, flags)
    if record:
        workspace = Workspace()
    elif workspace is None:
        workspace = _default_workspace("multi", y.device, stream)
    ws_ptr, ws_len = workspace.get(nbytes, y.device, stream)
    if out is None:
        out = torch.empty((B, n * P, N, M), dtype=torch.float32, device=y.device)
    elif out.shape != (B, n * P, N, M) or not out.is_contiguous():
        raise ValueError("out must be a contiguous (B, n*P, N, M) float32 tensor")
    lp, rp = _ptr_array([d.lam for d in dv]), _ptr_array([d.rho for d in dv])
    _lib.check(_lib.load().admm_tvd_forward_multi_dev_f32(y4.data_ptr(), out.data_ptr(), M, N, P, B, n, lp, rp,
                                                          int(maxit), flags, ws_ptr, ws_len, s_handle))
    if not record:
        return out
    rec = MultiRecording()
    rec.workspace, rec.dims, rec.maxit, rec.masks, rec.dv = (workspace, (M, N, P, B, n), int(maxit),
                                                             not need_rho or isotropic, dv)
    return out, rec


def tvd_fft_multi_backward_recorded(rec, x, x_bar, *, need_y=True, need_rho=True, stream=None):
    """Reverse sweep of a recorded multi-branch forward (x = its output, unmodified; x_bar in x's chcat
    layout).  Returns (y_bar or None, lam_bar (n,), rho_bar (n,) or None); y_bar sums the branches' input
    gradients.  Consumes the recording."""
    if rec.workspace is None:
        raise RuntimeError("recording already consumed")
    M, N, P, B, n = rec.dims
    if need_rho and rec.masks:
        raise ValueError("recorded with need_rho=False: rho_bar is not available")
    stream, s_handle = _stream_of(stream, x.device)
    xb = x_bar.reshape(x.shape).to(torch.float32).contiguous()
    ws_ptr, ws_len = rec.workspace.get(0, x.device, stream)
    y_bar = torch.empty((B, P, N, M), dtype=torch.float32, device=x.device) if need_y else None
    scal = torch.zeros(2 * n, dtype=torch.float32, device=x.device)
    _lib.check(_lib.load().admm_tvd_backward_multi_recorded_dev_f32(
        xb.data_ptr(), y_bar.data_ptr() if need_y else None, scal.data_ptr(),
        scal.data_ptr() + 4 * n if need_rho else None, M, N, P, B, n, rec.maxit, x.data_ptr(), ws_ptr, ws_len,
        s_handle))
    rec.workspace = None
    return y_bar, scal[:n], scal[n:] if need_rho else None


class _TvdFFTMultiFn(torch.autograd.Function):
    """Differentiable tvd_fft_multi: one recorded forward of every branch, one reverse sweep."""

    @staticmethod
    def forward(ctx, y, maxit, iso, n, *params):
        lams, rhos = params[:n], params[n:]
        ctx.n = n
        need_rho = any(ctx.needs_input_grad[4 + n + i] for i in range(n))
        if iso and need_rho:
            raise NotImplementedError("rho_bar of the isotropic multi-branch solve: solve the branches one by one")
        x, ctx.rec = tvd_fft_multi(y, lams, rhos, maxit, record=True, need_rho=need_rho, isotropic=iso)
        ctx.need_rho = need_rho
        ctx.save_for_backward(y, x, *params)
        return x

    @staticmethod
    def backward(ctx, x_bar):
        y, x, *params = ctx.saved_tensors
        n = ctx.n
        yb, lb, rb = tvd_fft_multi_backward_recorded(ctx.rec, x, x_bar, need_y=ctx.needs_input_grad[0],
                                                     need_rho=ctx.need_rho)
        ctx.rec = None
        grads = [yb if ctx.needs_input_grad[0] else None, None, None, None]
        for i in range(n):
            p = params[i]
            grads.append(lb[i:i + 1].reshape(p.shape).to(p.dtype) if ctx.needs_input_grad[4 + i] else None)
        for i in range(n):
            p = params[n + i]
            grads.append(rb[i:i + 1].reshape(p.shape).to(p.dtype) if ctx.needs_input_grad[4 + n + i] else None)
        return tuple(grads)


def tvd_fft_multi_grad(y, lams, rhos, maxit=100, isotropic=False):
    """tvd_fft_multi under autograd when y or any lam / rho tensor requires grad (else the plain call)."""
    ts = [t for t in (y, *lams, *rhos) if isinstance(t, torch.Tensor)]
    if torch.is_grad_enabled() and any(t.requires_grad for t in ts):
        dev = y.device
        as_t = lambda v: v if isinstance(v, torch.Tensor) else torch.full((1,), float(v), device=dev)  # noqa: E731
        return _TvdFFTMultiFn.apply(y, int(maxit), bool(isotropic), len(lams), *[as_t(v) for v in lams],
                                    *[as_t(v) for v in rhos])
    return tvd_fft_multi(y, lams, rhos, maxit, isotropic=isotropic)
