"""Device-level unit tests of the fused-kernel building blocks (libadmm_devtest.so).

The lane-pair (line_pair.hpp) and lane-quad (line_quad.hpp) line transforms against numpy's rFFT (packed half spectrum: slot 0 =
(X[0], X[M/2]), the convention of the 2-pass kernels and tests/kernel_model.py).
"""
import ctypes
import os

import numpy as np
import pytest

from conftest import PKG_DIR

pytestmark = pytest.mark.gpu


def _lib():
    path = os.path.join(PKG_DIR, "libadmm_devtest.so")
    if not os.path.exists(path):
        pytest.fail("libadmm_devtest.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    for fn in ("devtest_pair_forward", "devtest_pair_inverse", "devtest_quad_forward", "devtest_quad_inverse"):
        getattr(lib, fn).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        getattr(lib, fn).restype = ctypes.c_int
    return lib


def pack(X):
    P = X[..., :128].copy()
    P[..., 0] = X[..., 0].real + 1j * X[..., 128].real
    return P


@pytest.mark.parametrize("layout", ["pair", "quad"])
def test_line_forward_inverse(dev, layout):
    import torch
    lib = _lib()
    fwd, inv = getattr(lib, f"devtest_{layout}_forward"), getattr(lib, f"devtest_{layout}_inverse")
    rng = np.random.default_rng(3)
    rows = 512
    x = rng.standard_normal((rows, 256)).astype(np.float32)
    xt = torch.from_numpy(x).to(dev)
    spec = torch.zeros((rows, 128), dtype=torch.complex64, device=dev)
    assert fwd(xt.data_ptr(), spec.data_ptr(), rows) == 0
    want = pack(np.fft.rfft(x.astype(np.float64), axis=-1))
    got = spec.cpu().numpy()
    err = np.abs(got - want).max() / np.abs(want).max()
    assert err < 2e-6, err

    # inverse of an arbitrary packed spectrum: 256 * irfft
    X = (rng.standard_normal((rows, 129)) + 1j * rng.standard_normal((rows, 129)))
    X[:, 0] = X[:, 0].real
    X[:, 128] = X[:, 128].real
    Pk = pack(X).astype(np.complex64)
    st = torch.from_numpy(Pk).to(dev)
    out = torch.zeros((rows, 256), dtype=torch.float32, device=dev)
    assert inv(st.data_ptr(), out.data_ptr(), rows) == 0
    want = 256.0 * np.fft.irfft(X, n=256, axis=-1)
    err = np.abs(out.cpu().numpy() - want).max() / np.abs(want).max()
    assert err < 2e-6, err
