"""GPU: replay every `ccall` of julia/ADMMDeconvHIP.jl through ctypes, typed by the shim's own type tuples
(tests/julia_abi.py parses them) and with the shim's argument lists: λ / ρ as device pointers, C_NULL
with kh = kw = 0 for the empty PSF, the 256-byte aligned workspace pointer, `pointer(scal) + 4` for ρ̄,
the stream handle and a C_NULL reducer.  Results must be bitwise those of the Python binding (which the
parity tests check against the oracle).  Julia itself is absent; this is the closest executable check
of the binding a maintainer would add (/root/reference/src/ops/ops.jl:181)."""
import ctypes

import numpy as np
import pytest
import torch

import admm_deconv
from admm_deconv import _lib, synth
from julia_abi import ctypes_function, julia_ccalls

pytestmark = pytest.mark.gpu

CALLS = julia_ccalls()
LAM, RHO = 0.0041, 0.021


def _fn(name):
    return ctypes_function(_lib.load(), name, CALLS[name])


def _ws(nbytes, dev):
    buf = torch.empty(nbytes + 256, dtype=torch.uint8, device=dev)
    p = buf.data_ptr()
    off = (256 - p % 256) % 256
    return buf, p + off, buf.numel() - off


@pytest.mark.parametrize("psf", [False, True], ids=["empty-psf", "psf"])
@pytest.mark.parametrize("shape", [(2, 1, 256, 256), (1, 3, 64, 48)], ids=["fused", "generic-rgb"])
def test_forward_ccall_replay(dev, psf, shape):
    B, P, N, M = shape
    h = synth.gaussian_psf(7, 1.3) if psf else None
    y = torch.from_numpy(synth.make_batch(B, M, N, h, P=P)).to(dev)
    hd = torch.from_numpy(h).to(dev) if psf else None
    kh, kw = (7, 7) if psf else (0, 0)
    lam = torch.tensor([LAM], dtype=torch.float32, device=dev)      # _dev32(λ): Float32 ROCArray
    rho = torch.tensor([RHO], dtype=torch.float64, device=dev).float()   # Float64 λ/ρ narrowed on device
    nbytes = ctypes.c_size_t(0)
    assert _fn("admm_tvd_workspace_bytes")(M, N, P, B, kh, kw, 0, ctypes.byref(nbytes)) == 0
    buf, ws, wslen = _ws(nbytes.value, dev)
    x = torch.empty_like(y)
    s = torch.cuda.current_stream(dev).cuda_stream
    rc = _fn("admm_tvd_forward_dev_f32")(y.data_ptr(), x.data_ptr(), M, N, P, B, hd.data_ptr() if psf else None,
                                         kh, kw, lam.data_ptr(), rho.data_ptr(), 0, 12, ws, wslen, s, None)
    assert rc == 0, _lib.load().admm_last_error()
    ref = admm_deconv.tvd_fft(y, LAM, RHO, hd, False, 12)
    torch.cuda.synchronize()
    assert torch.equal(x, ref)


@pytest.mark.parametrize("psf", [False, True], ids=["empty-psf", "psf"])
def test_rrule_ccall_replay(dev, psf):
    """The rrule: record (want_h = !isempty(h)) then the pullback's reverse sweep with (λ̄, ρ̄) written to
    pointer(scal) and pointer(scal) + 4."""
    B, P, N, M, K = 2, 1, 256, 256, 9
    h = synth.gaussian_psf(5, 1.0) if psf else None
    y = torch.from_numpy(synth.make_batch(B, M, N, h, g0=4)).to(dev)
    hd = torch.from_numpy(h).to(dev) if psf else None
    kh, kw = (5, 5) if psf else (0, 0)
    want_h = int(psf)
    lam = torch.tensor([LAM], device=dev)
    rho = torch.tensor([RHO], device=dev)
    xb = torch.randn_like(y)
    nbytes = ctypes.c_size_t(0)
    assert _fn("admm_tvd_backward_workspace_bytes")(M, N, P, B, kh, kw, 0, K, want_h, ctypes.byref(nbytes)) == 0
    buf, ws, wslen = _ws(nbytes.value, dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    x = torch.empty_like(y)
    hp = hd.data_ptr() if psf else None
    rc = _fn("admm_tvd_forward_record_dev_f32")(y.data_ptr(), x.data_ptr(), M, N, P, B, hp, kh, kw, lam.data_ptr(),
                                                rho.data_ptr(), 0, K, want_h, ws, wslen, s, None)
    assert rc == 0, _lib.load().admm_last_error()
    yb = torch.empty_like(y)
    hb = torch.empty_like(hd) if psf else None
    scal = torch.zeros(2, dtype=torch.float32, device=dev)
    rc = _fn("admm_tvd_backward_recorded_dev_f32")(
        y.data_ptr(), xb.data_ptr(), yb.data_ptr(), hb.data_ptr() if psf else None, scal.data_ptr(),
        scal.data_ptr() + 4, M, N, P, B, hp, kh, kw, lam.data_ptr(), rho.data_ptr(), 0, K, x.data_ptr(), ws, wslen,
        s, None)
    assert rc == 0, _lib.load().admm_last_error()
    x2, yb2, hb2, lb2, rb2 = admm_deconv.tvd_fft_backward(y, xb, LAM, RHO, hd, False, K, need_h=psf)
    torch.cuda.synchronize()
    assert torch.equal(x, x2) and torch.equal(yb, yb2)
    assert torch.equal(scal[0], lb2) and torch.equal(scal[1], rb2)
    if psf:
        assert torch.equal(hb, hb2)
    assert np.isfinite(scal.cpu().numpy()).all()
