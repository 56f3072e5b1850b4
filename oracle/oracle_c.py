"""ctypes wrapper for the C oracle (oracle/_build/liboracle.so) -- TEST INFRASTRUCTURE ONLY.

Used by tests/ (fp64 cross-check of oracle_np.py) and by bench.py's `cpu_baseline` leg, which
times `oracle_tvd_fft_f32` (the op-for-op C restatement of /root/reference/src/ops/ops.jl:17-96
in the reference's own Float32) on the host cores.  Parity unpinned: see oracle_np.py.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        for name, ct in (("oracle_tvd_fft_f32", ctypes.c_float), ("oracle_tvd_fft_f64", ctypes.c_double)):
            f = getattr(L, name)
            f.restype = ctypes.c_int
            f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                          ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ct, ct,
                          ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.oracle_max_threads.restype = ctypes.c_int
        _lib = L
    return _lib


def max_threads():
    return lib().oracle_max_threads()


def tvd_fft_c(y_c, lam, rho, h_c=None, iso=False, maxit=100, dtype=np.float32, nthreads=0):
    """C-layout entry: y_c (B,P,N,M), h_c (kw,kh) numpy arrays.  Returns x_c (B,P,N,M)."""
    dtype = np.dtype(dtype)
    fn = lib().oracle_tvd_fft_f32 if dtype == np.float32 else lib().oracle_tvd_fft_f64
    y = np.ascontiguousarray(y_c, dtype=dtype)
    B, P, N, M = y.shape
    x = np.empty_like(y)
    if h_c is None or np.size(h_c) == 0:
        hp, kh, kw, hbuf = None, 0, 0, None
    else:
        hbuf = np.ascontiguousarray(h_c, dtype=dtype)
        kw, kh = hbuf.shape
        hp = hbuf.ctypes.data
    rc = fn(y.ctypes.data, x.ctypes.data, M, N, P, B, hp, kh, kw, float(lam), float(rho),
            int(bool(iso)), int(maxit), int(nthreads))
    if rc != 0:
        raise ValueError(f"oracle_tvd_fft failed rc={rc}")
    return x
