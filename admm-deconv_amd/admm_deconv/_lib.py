"""ctypes binding of the C ABI declared in include/admm_deconv.h.

The product path: every solve goes through `libadmm_deconv.so` (hand-written HIP for gfx950).
There is no CPU or PyTorch fallback -- if the library is missing, loading fails loudly.
"""
from __future__ import annotations

import ctypes
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))   # .../admm-deconv_amd
# ADMM_LIB_PATH: another build of the library for A/B timing experiments (tools/); default the in-tree build
LIB_PATH = os.environ.get("ADMM_LIB_PATH") or os.path.join(PKG_ROOT, "libadmm_deconv.so")

ADMM_OK = 0
ADMM_E_INVALID = -1
ADMM_E_UNSUPPORTED = -2
ADMM_E_WORKSPACE = -3
ADMM_E_HIP = -4
ADMM_E_REDUCER = -5

# library options (admm_set_option, include/admm_deconv.h)
OPT_FUSED, OPT_FUSED_ADJ, OPT_LINE_T, OPT_COL_THREADS, OPT_GEN_TM, OPT_GEN_KN, OPT_PLANE_STAGGER, OPT_SMOOTH, OPT_RESIDENT, \
    OPT_MIN_PLANES, OPT_MALL_STREAMS = range(11)
OPTIONS = {"FUSED": OPT_FUSED, "FUSED_ADJ": OPT_FUSED_ADJ, "LINE_T": OPT_LINE_T, "COL_THREADS": OPT_COL_THREADS,
           "GEN_TM": OPT_GEN_TM, "GEN_KN": OPT_GEN_KN, "PLANE_STAGGER": OPT_PLANE_STAGGER,
           "SMOOTH": OPT_SMOOTH, "RESIDENT": OPT_RESIDENT, "MIN_PLANES": OPT_MIN_PLANES,
           "MALL_STREAMS": OPT_MALL_STREAMS}

K_SETUP, K_PREP, K_COLUMN, K_LINE, K_FINAL, K_NORM, K_PLANE, K_ADJ = range(8)
KERNEL_CLASSES = {K_SETUP: "setup", K_PREP: "prep", K_COLUMN: "column", K_LINE: "line",
                  K_FINAL: "final", K_NORM: "norm", K_PLANE: "plane", K_ADJ: "adjoint"}

# Every symbol include/admm_deconv.h declares (checked by tests/test_capi.py).
EXPORTS = ("admm_abi_version", "admm_last_error", "admm_tvd_workspace_bytes", "admm_tvd_forward_f32",
           "admm_tvd_backward_workspace_bytes", "admm_tvd_backward_f32",
           "admm_tvd_forward_sharded_f32", "admm_tvd_backward_sharded_f32",
           "admm_tvd_forward_record_f32", "admm_tvd_backward_recorded_f32",
           "admm_tvd_forward_dev_f32", "admm_tvd_backward_dev_f32", "admm_tvd_forward_record_dev_f32",
           "admm_tvd_backward_recorded_dev_f32", "admm_set_option", "admm_get_option",
           "admm_metrics_workspace_bytes", "admm_gmsd_f32", "admm_gmsd_backward_f32", "admm_ssim_f32", "admm_mse_f32",
           "admm_profile_enable", "admm_profile_reset", "admm_profile_get",
           "admm_tvd_multi_workspace_bytes", "admm_tvd_forward_multi_dev_f32",
           "admm_tvd_backward_multi_recorded_dev_f32", "admm_copy_async", "admm_query_paths", "admm_query_forward_schedule", "admm_clamp_backward_f32",
           "admm_path_name", "admm_ipc_get_handle", "admm_ipc_open", "admm_ipc_close")

# record flags (the want_hbar word of the record entry points) and multi-branch flags
REC_HBAR, REC_MASKS = 1, 2
MULTI_RECORD, MULTI_ISO = 1, 4


# admm_reduce_fn / admm_batch_reducer (include/admm_deconv.h): cross-shard sum of an M x N map
REDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p)


class BatchReducer(ctypes.Structure):
    _fields_ = [("fn", REDUCE_FN), ("user", ctypes.c_void_p)]


class AdmmError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"admm_deconv error {code}: {msg}")
        self.code = code


_lib = None


def load():
    """Load the in-tree HIP library (built by __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                          "(there is deliberately no CPU fallback)")
    try:
        import torch  # noqa: F401  -- share torch's HIP runtime (same SONAME) when torch is in use
    except Exception:
        pass
    L = ctypes.CDLL(LIB_PATH)
    c_int, c_float, c_size_t, c_void_p = ctypes.c_int, ctypes.c_float, ctypes.c_size_t, ctypes.c_void_p
    L.admm_abi_version.restype = c_int
    L.admm_abi_version.argtypes = []
    L.admm_last_error.restype = ctypes.c_char_p
    L.admm_last_error.argtypes = []
    L.admm_tvd_workspace_bytes.restype = c_int
    L.admm_tvd_workspace_bytes.argtypes = [c_int] * 7 + [ctypes.POINTER(c_size_t)]
    L.admm_tvd_forward_f32.restype = c_int
    L.admm_tvd_forward_f32.argtypes = [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int,
                                       c_float, c_float, c_int, c_int, c_void_p, c_size_t, c_void_p]
    L.admm_tvd_backward_workspace_bytes.restype = c_int
    L.admm_tvd_backward_workspace_bytes.argtypes = [c_int] * 9 + [ctypes.POINTER(c_size_t)]
    L.admm_tvd_backward_f32.restype = c_int
    L.admm_tvd_backward_f32.argtypes = [c_void_p] * 6 + [c_int] * 4 + [c_void_p, c_int, c_int, c_float, c_float,
                                                                         c_int, c_int, c_void_p, c_void_p, c_size_t,
                                                                         c_void_p]
    L.admm_tvd_forward_sharded_f32.restype = c_int
    L.admm_tvd_forward_sharded_f32.argtypes = list(L.admm_tvd_forward_f32.argtypes) + [ctypes.POINTER(BatchReducer)]
    L.admm_tvd_backward_sharded_f32.restype = c_int
    L.admm_tvd_backward_sharded_f32.argtypes = list(L.admm_tvd_backward_f32.argtypes) + [ctypes.POINTER(BatchReducer)]
    L.admm_tvd_forward_record_f32.restype = c_int
    L.admm_tvd_forward_record_f32.argtypes = [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int,
                                              c_float, c_float, c_int, c_int, c_int, c_void_p, c_size_t, c_void_p,
                                              ctypes.POINTER(BatchReducer)]
    L.admm_tvd_backward_recorded_f32.restype = c_int
    L.admm_tvd_backward_recorded_f32.argtypes = list(L.admm_tvd_backward_sharded_f32.argtypes)
    # device-resident lambda / rho (include/admm_deconv.h): same argument lists with two device pointers
    # in place of the two floats, and a (nullable) reducer at the end
    L.admm_tvd_forward_dev_f32.restype = c_int
    L.admm_tvd_forward_dev_f32.argtypes = [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int,
                                           c_void_p, c_void_p, c_int, c_int, c_void_p, c_size_t, c_void_p,
                                           ctypes.POINTER(BatchReducer)]
    L.admm_tvd_backward_dev_f32.restype = c_int
    L.admm_tvd_backward_dev_f32.argtypes = [c_void_p] * 6 + [c_int] * 4 + [c_void_p, c_int, c_int, c_void_p, c_void_p,
                                                                             c_int, c_int, c_void_p, c_void_p, c_size_t,
                                                                             c_void_p, ctypes.POINTER(BatchReducer)]
    L.admm_tvd_forward_record_dev_f32.restype = c_int
    L.admm_tvd_forward_record_dev_f32.argtypes = [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int,
                                                  c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_size_t,
                                                  c_void_p, ctypes.POINTER(BatchReducer)]
    L.admm_tvd_backward_recorded_dev_f32.restype = c_int
    L.admm_tvd_backward_recorded_dev_f32.argtypes = list(L.admm_tvd_backward_dev_f32.argtypes)
    L.admm_tvd_multi_workspace_bytes.restype = c_int
    L.admm_tvd_multi_workspace_bytes.argtypes = [c_int] * 7 + [ctypes.POINTER(c_size_t)]
    L.admm_tvd_forward_multi_dev_f32.restype = c_int
    L.admm_tvd_forward_multi_dev_f32.argtypes = [c_void_p, c_void_p] + [c_int] * 5 + [
        ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p), c_int, c_int, c_void_p, c_size_t, c_void_p]
    L.admm_tvd_backward_multi_recorded_dev_f32.restype = c_int
    L.admm_tvd_backward_multi_recorded_dev_f32.argtypes = [c_void_p] * 4 + [c_int] * 6 + [c_void_p, c_void_p,
                                                                                          c_size_t, c_void_p]
    L.admm_set_option.restype = c_int
    L.admm_set_option.argtypes = [c_int, c_int]
    L.admm_get_option.restype = c_int
    L.admm_get_option.argtypes = [c_int, ctypes.POINTER(c_int)]
    L.admm_metrics_workspace_bytes.restype = c_int
    L.admm_metrics_workspace_bytes.argtypes = [c_int] * 6 + [ctypes.POINTER(c_size_t)]
    L.admm_gmsd_f32.restype = c_int
    L.admm_gmsd_f32.argtypes = [c_void_p, c_void_p] + [c_int] * 4 + [c_float, c_float, c_void_p, c_void_p, c_void_p,
                                                                     c_void_p, c_size_t, c_void_p]
    L.admm_gmsd_backward_f32.restype = c_int
    L.admm_gmsd_backward_f32.argtypes = [c_void_p, c_void_p] + [c_int] * 4 + [c_float, c_float, c_void_p, c_void_p,
                                                                              c_void_p, c_size_t, c_void_p]
    L.admm_ssim_f32.restype = c_int
    L.admm_ssim_f32.argtypes = [c_void_p, c_void_p] + [c_int] * 4 + [ctypes.POINTER(c_float), c_int, c_float, c_int,
                                                                     c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                                                     c_void_p]
    L.admm_mse_f32.restype = c_int
    L.admm_mse_f32.argtypes = [c_void_p, c_void_p] + [c_int] * 4 + [c_void_p, c_void_p, c_size_t, c_void_p]
    L.admm_profile_enable.restype = c_int
    L.admm_profile_enable.argtypes = [c_int]
    L.admm_profile_reset.restype = c_int
    L.admm_profile_reset.argtypes = []
    L.admm_profile_get.restype = c_int
    L.admm_profile_get.argtypes = [c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_longlong)]
    L.admm_copy_async.restype = c_int
    L.admm_copy_async.argtypes = [c_void_p, c_void_p, c_size_t, c_void_p]
    L.admm_ipc_get_handle.restype = c_int
    L.admm_ipc_get_handle.argtypes = [c_void_p, c_void_p, ctypes.POINTER(c_size_t)]
    L.admm_ipc_open.restype = c_int
    L.admm_ipc_open.argtypes = [c_void_p, c_int, ctypes.POINTER(c_void_p)]
    L.admm_ipc_close.restype = c_int
    L.admm_ipc_close.argtypes = [c_void_p, c_int]
    L.admm_query_paths.restype = c_int
    L.admm_query_paths.argtypes = [c_int] * 4 + [ctypes.c_longlong] + [c_int] * 4 + [ctypes.POINTER(c_int)] * 2
    L.admm_clamp_backward_f32.restype = c_int
    L.admm_clamp_backward_f32.argtypes = [c_void_p, c_void_p, c_void_p, c_size_t, c_float, c_float, c_void_p]
    L.admm_query_forward_schedule.restype = c_int
    L.admm_query_forward_schedule.argtypes = [c_int] * 4 + [ctypes.c_longlong, ctypes.POINTER(ctypes.c_longlong),
                                              ctypes.POINTER(c_int)]
    L.admm_path_name.restype = ctypes.c_char_p
    L.admm_path_name.argtypes = [c_int]
    _lib = L
    return L


def check(rc):
    if rc != ADMM_OK:
        raise AdmmError(rc, load().admm_last_error().decode(errors="replace"))
    return rc


def workspace_bytes(M, N, P, B, kh, kw, iso):
    out = ctypes.c_size_t(0)
    check(load().admm_tvd_workspace_bytes(M, N, P, B, kh, kw, int(bool(iso)), ctypes.byref(out)))
    return out.value


def backward_workspace_bytes(M, N, P, B, kh, kw, iso, maxit, want_hbar):
    """want_hbar: a bool (h_bar wanted) or the flag word REC_HBAR | REC_MASKS."""
    out = ctypes.c_size_t(0)
    flags = int(want_hbar)
    check(load().admm_tvd_backward_workspace_bytes(M, N, P, B, kh, kw, int(bool(iso)), int(maxit), flags,
                                                   ctypes.byref(out)))
    return out.value


def multi_workspace_bytes(M, N, P, B, nbranch, maxit, flags):
    out = ctypes.c_size_t(0)
    check(load().admm_tvd_multi_workspace_bytes(M, N, P, B, nbranch, int(maxit), int(flags), ctypes.byref(out)))
    return out.value


MODE_FORWARD, MODE_RECORD, MODE_BACKWARD = 0, 1, 2


def query_paths(M, N, iso=False, kh=0, mode=MODE_FORWARD, flags=0, want_hbar=False, want_rho=False, planes=0):
    """admm_query_paths: (forward path name, reverse-sweep path name or None) the library would run for a call
    of `planes` = P * B planes (0: no plane-count rule, OPT_MIN_PLANES)."""
    L = load()
    f, b = ctypes.c_int(0), ctypes.c_int(0)
    check(L.admm_query_paths(M, N, int(iso), kh, int(planes), mode, flags, int(want_hbar), int(want_rho),
                             ctypes.byref(f), ctypes.byref(b)))
    return L.admm_path_name(f.value).decode(), (L.admm_path_name(b.value).decode() if b.value else None)


def forward_schedule(M, N, iso=False, kh=0, planes=1):
    """admm_query_forward_schedule: (planes per launch, streams) of a forward over `planes` planes."""
    c, n = ctypes.c_longlong(0), ctypes.c_int(0)
    check(load().admm_query_forward_schedule(M, N, int(iso), kh, int(planes), ctypes.byref(c), ctypes.byref(n)))
    return c.value, n.value


def copy_async(dst, src, nbytes, stream):
    """admm_copy_async: hipMemcpyAsync of nbytes between device pointers on a HIP stream handle (int)."""
    check(load().admm_copy_async(dst, src, nbytes, stream))


IPC_HANDLE_BYTES = 64


def ipc_get_handle(ptr):
    """admm_ipc_get_handle: (handle bytes, byte offset of ptr in its allocation)."""
    buf = ctypes.create_string_buffer(IPC_HANDLE_BYTES)
    off = ctypes.c_size_t(0)
    check(load().admm_ipc_get_handle(ptr, buf, ctypes.byref(off)))
    return buf.raw, off.value


def ipc_open(handle, device):
    """admm_ipc_open: map a peer's allocation on this process's `device`; returns its base address (int)."""
    if len(handle) != IPC_HANDLE_BYTES:
        raise ValueError("IPC handle must be 64 bytes")
    p = ctypes.c_void_p(0)
    check(load().admm_ipc_open(handle, int(device), ctypes.byref(p)))
    return int(p.value)


def ipc_close(ptr, device):
    check(load().admm_ipc_close(ptr, int(device)))


def profile_enable(on=True):
    check(load().admm_profile_enable(int(bool(on))))


def profile_reset():
    check(load().admm_profile_reset())


def profile_get(cls):
    ms = ctypes.c_double(0)
    n = ctypes.c_longlong(0)
    check(load().admm_profile_get(int(cls), ctypes.byref(ms), ctypes.byref(n)))
    return ms.value, n.value


def set_option(opt, value):
    """admm_set_option: `opt` is an OPT_* index or a name from OPTIONS ("FUSED", "LINE_T", ...)."""
    check(load().admm_set_option(OPTIONS[opt] if isinstance(opt, str) else int(opt), int(value)))


def get_option(opt):
    v = ctypes.c_int(0)
    check(load().admm_get_option(OPTIONS[opt] if isinstance(opt, str) else int(opt), ctypes.byref(v)))
    return v.value


class option:
    """Context manager: `with option("FUSED", 0): ...` sets a library option and restores it."""

    def __init__(self, opt, value):
        self.opt, self.value = opt, value

    def __enter__(self):
        self.old = get_option(self.opt)
        set_option(self.opt, self.value)
        return self

    def __exit__(self, *a):
        set_option(self.opt, self.old)
