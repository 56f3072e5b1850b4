"""CPU: the C-ABI library loads, exports every symbol include/*.h declares, and validates
arguments (no GPU compute is issued by these calls)."""
import ctypes
import os
import re

import pytest

from admm_deconv import _lib

INC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
HDRS = [os.path.join(INC, f) for f in ("admm_deconv.h", "admm_metrics.h")]


def header_functions():
    names = set()
    for h in HDRS:
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"\b(admm_\w+)\s*\(", src))
    names.discard("admm_reduce_fn")   # the reducer callback typedef, not an export
    return sorted(names)


def test_header_and_binding_agree():
    assert header_functions() == sorted(_lib.EXPORTS)


def test_library_exports_every_symbol():
    L = _lib.load()
    for name in header_functions():
        assert hasattr(L, name), name
    assert L.admm_abi_version() == 3


def test_workspace_bytes():
    n1 = _lib.workspace_bytes(256, 256, 1, 512, 15, 15, False)
    n0 = _lib.workspace_bytes(256, 256, 1, 512, 0, 0, False)
    assert n1 > n0 >= 512 * 256 * 256 * 4 * 6
    assert _lib.workspace_bytes(256, 256, 1, 512, 15, 15, True) > n1


def test_workspace_sized_for_one_chunk_of_planes():
    """Aniso batches above 65,280 planes run as consecutive chunks through one chunk-sized workspace
    (include/admm_deconv.h); iso (batch-coupled) and the adjoint keep the 65535-plane limit."""
    chunk = 255 * 256
    assert _lib.workspace_bytes(8, 8, 1, 200000, 3, 3, False) == _lib.workspace_bytes(8, 8, 1, chunk, 3, 3, False)
    assert _lib.workspace_bytes(8, 8, 1, chunk, 3, 3, False) > _lib.workspace_bytes(8, 8, 1, chunk - 256, 3, 3, False)
    out = ctypes.c_size_t(0)
    L = _lib.load()
    assert L.admm_tvd_workspace_bytes(8, 8, 1, 70000, 3, 3, 1, ctypes.byref(out)) == _lib.ADMM_E_UNSUPPORTED
    assert L.admm_tvd_backward_workspace_bytes(8, 8, 1, 70000, 3, 3, 0, 5, 0, ctypes.byref(out)) == \
        _lib.ADMM_E_UNSUPPORTED
    assert "65535" in L.admm_last_error().decode()


def test_isotropic_batch_is_never_chunked():
    """The isotropic prox couples the whole batch (ops.jl:6): a batch above one anisotropic chunk (65,280
    planes) but within the isotropic limit (65,535) is sized -- and solved -- as ONE launch sequence."""
    chunk = 255 * 256
    iso = [_lib.workspace_bytes(4, 4, 1, n, 0, 0, True) for n in (chunk, 65300, 65535)]
    assert iso[0] < iso[1] < iso[2]
    assert _lib.workspace_bytes(4, 4, 1, 65300, 0, 0, False) == _lib.workspace_bytes(4, 4, 1, chunk, 0, 0, False)


def test_mall_resident_schedule():
    """ADMM_OPT_MALL_STREAMS (admm_paths.hip forward_chunks): an anisotropic 2-pass batch whose 28 B/px per-iteration
    set exceeds 512 MiB runs as ~224 MiB / n chunks on n streams, with one chunk workspace per stream; c4 (768
    planes of 512^2) is 8 planes x 4 streams.  Smaller batches, chunks under 4 planes, isotropic batches and the
    one-workgroup-per-plane paths are one stream."""
    assert _lib.get_option("MALL_STREAMS") == 4
    assert _lib.forward_schedule(512, 512, False, 15, 768) == (8, 4)
    assert _lib.forward_schedule(512, 512, False, 15, 60) == (60, 1)         # 420 MB: one stream
    assert _lib.forward_schedule(512, 512, True, 15, 768) == (768, 1)        # the prox couples the batch
    assert _lib.forward_schedule(1024, 1024, False, 0, 64) == (64, 1)       # 2-plane chunks would lose
    assert _lib.forward_schedule(640, 480, False, 15, 64) == (6, 4)          # the smooth-length kernels too
    assert _lib.forward_schedule(250, 250, False, 15, 256)[1] == 1           # the CU-resident path
    assert _lib.forward_schedule(256, 256, False, 15, 4096)[1] == 1          # the fused path
    w4 = _lib.workspace_bytes(512, 512, 3, 256, 15, 15, False)
    with _lib.option("MALL_STREAMS", 1):
        assert _lib.forward_schedule(512, 512, False, 15, 768) == (768, 1)
        w1 = _lib.workspace_bytes(512, 512, 3, 256, 15, 15, False)
        one = _lib.workspace_bytes(512, 512, 1, 8, 15, 15, False)
    with _lib.option("MALL_STREAMS", 2):
        assert _lib.forward_schedule(512, 512, False, 15, 768) == (16, 2)
    assert w4 >= 4 * one and w4 < 4 * one + 4 * 4096 and w4 < w1 / 20
    L = _lib.load()
    c, n = ctypes.c_longlong(0), ctypes.c_int(0)
    assert L.admm_query_forward_schedule(512, 512, 0, 15, 0, ctypes.byref(c), ctypes.byref(n)) == _lib.ADMM_E_INVALID
    assert L.admm_query_forward_schedule(512, 512, 0, 15, 8, None, ctypes.byref(n)) == _lib.ADMM_E_INVALID


@pytest.mark.parametrize("args,code", [
    ((8192, 64, 1, 1, 5, 5, 0), _lib.ADMM_E_UNSUPPORTED),  # M too large
    ((64, 8192, 1, 1, 5, 5, 0), _lib.ADMM_E_UNSUPPORTED),  # N too large
    ((1, 64, 1, 1, 0, 0, 0), _lib.ADMM_E_UNSUPPORTED),     # M < 2 (ops.jl:33 needs a second row)
    ((64, 1, 1, 1, 0, 0, 0), _lib.ADMM_E_UNSUPPORTED),     # N < 2
    ((64, 64, 1, 1, 5, 0, 0), _lib.ADMM_E_INVALID),        # half-empty PSF
    ((64, 64, 0, 1, 5, 5, 0), _lib.ADMM_E_INVALID),        # P = 0
    ((64, 64, 1, 1, 65, 5, 0), _lib.ADMM_E_UNSUPPORTED),   # PSF taller than the image
])
def test_workspace_validation(args, code):
    out = ctypes.c_size_t(0)
    assert _lib.load().admm_tvd_workspace_bytes(*args, ctypes.byref(out)) == code
    assert len(_lib.load().admm_last_error()) > 0


def test_forward_argument_errors_before_any_device_work():
    L = _lib.load()
    fake = 1 << 20   # never dereferenced: validation fails first
    assert L.admm_tvd_forward_f32(None, fake, 64, 64, 1, 1, None, 0, 0, 0.1, 1.0, 0, 5, fake, 1 << 30, None) \
        == _lib.ADMM_E_INVALID
    assert L.admm_tvd_forward_f32(fake, fake, 64, 64, 1, 1, None, 0, 0, 0.1, 1.0, 0, -1, fake, 1 << 30, None) \
        == _lib.ADMM_E_INVALID
    assert L.admm_tvd_forward_f32(fake, fake, 64, 64, 1, 1, None, 0, 0, float("nan"), 1.0, 0, 5, fake, 1 << 30,
                                  None) == _lib.ADMM_E_INVALID
    assert L.admm_tvd_forward_f32(fake, fake, 64, 64, 1, 1, None, 0, 0, 0.1, 1.0, 0, 5, fake, 16, None) \
        == _lib.ADMM_E_WORKSPACE
    assert L.admm_tvd_forward_f32(fake, fake, 64, 64, 1, 1, None, 0, 0, 0.1, 1.0, 0, 5, fake + 8, 1 << 30, None) \
        == _lib.ADMM_E_WORKSPACE
    assert b"workspace" in L.admm_last_error()


def test_product_path_has_no_cpu_fallback():
    import torch
    from admm_deconv import tvd_fft
    with pytest.raises(TypeError):
        tvd_fft(torch.zeros(1, 1, 8, 8), 0.1, 1.0)


@pytest.mark.parametrize("M,N", [(48, 64), (100, 75), (37, 29), (64, 2048)])
def test_generic_shapes_workspace(M, N):
    """Shapes outside the power-of-two kernels run the runtime-length path, forward and adjoint."""
    out = ctypes.c_size_t(0)
    L = _lib.load()
    assert L.admm_tvd_workspace_bytes(M, N, 1, 2, 5, 5, 0, ctypes.byref(out)) == _lib.ADMM_OK
    assert out.value >= 2 * M * N * 4 * 4
    for iso in (0, 1):
        for want_h in (0, 1):
            assert L.admm_tvd_backward_workspace_bytes(M, N, 1, 2, 5, 5, iso, 4, want_h, ctypes.byref(out)) == _lib.ADMM_OK
            # trajectory (3 slots of s) + the dim-2 spectra when h_bar is wanted
            assert out.value >= 3 * 2 * 2 * M * N * 4 + want_h * 4 * 2 * (M // 2 + 1) * N * 8


def test_options_roundtrip_and_validation():
    """Library behaviour is switched by admm_set_option, never by the environment."""
    L = _lib.load()
    assert _lib.get_option("FUSED") == 1 and _lib.get_option("FUSED_ADJ") == 1
    with _lib.option("LINE_T", 4):
        assert _lib.get_option("LINE_T") == 4
    assert _lib.get_option("LINE_T") == 0
    assert L.admm_set_option(99, 1) == _lib.ADMM_E_INVALID
    assert L.admm_set_option(-1, 1) == _lib.ADMM_E_INVALID
    v = ctypes.c_int(0)
    assert L.admm_get_option(len(_lib.OPTIONS), ctypes.byref(v)) == _lib.ADMM_E_INVALID
    os.environ["ADMM_FUSED"] = "0"          # the round-1 environment knob is gone
    try:
        assert _lib.get_option("FUSED") == 1
    finally:
        del os.environ["ADMM_FUSED"]


def test_device_scalar_entry_points_validate():
    """The device-resident lambda / rho entry points (ops.jl:99,181 take 1-element device arrays) reject
    NULL scalar pointers before any device work."""
    L = _lib.load()
    fake = 1 << 20
    assert L.admm_tvd_forward_dev_f32(fake, fake, 64, 64, 1, 1, None, 0, 0, None, fake, 0, 5, fake, 1 << 30, None,
                                      None) == _lib.ADMM_E_INVALID
    assert L.admm_tvd_forward_record_dev_f32(fake, fake, 64, 64, 1, 1, None, 0, 0, fake, None, 0, 5, 0, fake,
                                             1 << 30, None, None) == _lib.ADMM_E_INVALID
    assert L.admm_tvd_backward_dev_f32(fake, fake, fake, None, None, None, 64, 64, 1, 1, None, 0, 0, None, None, 0,
                                       5, fake, fake, 1 << 30, None, None) == _lib.ADMM_E_INVALID
    assert b"device pointers" in L.admm_last_error()


def test_replay_without_recording_is_rejected():
    """A reverse sweep on a workspace that holds no recording fails with ADMM_E_INVALID (host-side
    check, before any device work)."""
    L = _lib.load()
    fake = 1 << 21   # 256-byte aligned, never dereferenced
    rc = L.admm_tvd_backward_recorded_f32(fake, fake, fake, None, None, None, 64, 64, 1, 1, None, 0, 0, 0.1, 1.0,
                                          0, 5, fake, fake, 1 << 34, None, None)
    assert rc == _lib.ADMM_E_INVALID
    assert b"no recording" in L.admm_last_error()


def test_backward_y_bar_optional_but_aligned():
    """y_bar may be NULL (input needs no gradient), but a given y_bar must be 16-byte aligned: rejected with
    ADMM_E_INVALID before any device work."""
    L = _lib.load()
    fake = 1 << 21
    rc = L.admm_tvd_backward_f32(fake, fake, fake + 4, None, None, None, 64, 64, 1, 1, None, 0, 0, 0.1, 1.0, 0, 5,
                                 fake, fake, 1 << 30, None)
    assert rc == _lib.ADMM_E_INVALID
    assert b"y_bar" in L.admm_last_error()


def test_multi_branch_workspace_and_validation():
    """admm_tvd_multi_workspace_bytes: the one-grid multi-branch solve covers 256 x 256 only, checks its
    flags, and a recording with ADMM_REC_MASKS needs far less trajectory memory than a full one."""
    L = _lib.load()
    out = ctypes.c_size_t(0)
    assert L.admm_tvd_multi_workspace_bytes(128, 128, 3, 2, 5, 10, 0, ctypes.byref(out)) == _lib.ADMM_E_UNSUPPORTED
    assert L.admm_tvd_multi_workspace_bytes(256, 256, 3, 2, 5, 10, 8, ctypes.byref(out)) == _lib.ADMM_E_INVALID
    assert L.admm_tvd_multi_workspace_bytes(256, 256, 3, 2, 0, 10, 0, ctypes.byref(out)) == _lib.ADMM_E_INVALID
    plain = _lib.multi_workspace_bytes(256, 256, 3, 64, 5, 50, 0)
    full = _lib.multi_workspace_bytes(256, 256, 3, 64, 5, 50, _lib.MULTI_RECORD)
    masks = _lib.multi_workspace_bytes(256, 256, 3, 64, 5, 50, _lib.MULTI_RECORD | _lib.REC_MASKS)
    planes, px = 5 * 3 * 64, 256 * 256
    assert full - plain >= 49 * planes * px * 8 and masks - plain < 49 * planes * px * 8 / 8
    # the single-solve recording with ADMM_REC_MASKS is sized for the mask trajectory too (from the fused
    # path's plane count on; 6 planes record for the 2-pass sweep, which takes no mask bits)
    f = _lib.backward_workspace_bytes(256, 256, 3, 32, 0, 0, False, 50, 0)
    m = _lib.backward_workspace_bytes(256, 256, 3, 32, 0, 0, False, 50, _lib.REC_MASKS)
    assert m < f
    assert _lib.backward_workspace_bytes(256, 256, 3, 2, 0, 0, False, 50, _lib.REC_MASKS) == \
        _lib.backward_workspace_bytes(256, 256, 3, 2, 0, 0, False, 50, 0)
    # isotropic (ADMM_MULTI_ISO): f maps and q partials on top of the plain layout; a recording keeps s_k
    # itself (the BT derivative needs it), |s_k| per branch and the R maps -- ADMM_REC_MASKS does not shrink it
    iso = _lib.multi_workspace_bytes(256, 256, 3, 64, 5, 50, _lib.MULTI_ISO)
    assert iso - plain >= 5 * px * 4 + planes * px * 4
    iso_rec = _lib.multi_workspace_bytes(256, 256, 3, 64, 5, 50, _lib.MULTI_ISO | _lib.MULTI_RECORD)
    assert iso_rec - full >= 49 * 5 * px * 4
    assert _lib.multi_workspace_bytes(256, 256, 3, 64, 5, 50, _lib.MULTI_ISO | _lib.MULTI_RECORD | _lib.REC_MASKS) == iso_rec
    # the single-solve isotropic recording without rho_bar (the fused sweep) keeps the full-size trajectory
    fi = _lib.backward_workspace_bytes(256, 256, 3, 2, 0, 0, True, 50, 0)
    assert _lib.backward_workspace_bytes(256, 256, 3, 2, 0, 0, True, 50, _lib.REC_MASKS) == fi


@pytest.mark.parametrize("iso", [False, True], ids=["aniso", "iso"])
def test_multi_branch_two_pass_layout(iso):
    """Below the fused paths' plane counts (96 aniso / 112 iso in all) the multi-branch workspace is the 2-pass
    kernels' (admm_capi.hip make_multi_layout two_pass: spectra, s state, natural-layout trajectory, per-branch
    maps and partial rows), from the rule's threshold on the fused kernels' (lane-native tables); MIN_PLANES = 0
    keeps the fused layout at every size.  c5 at batch 2 (5 x 6 planes) is below it."""
    fl = (_lib.MULTI_ISO if iso else 0)
    px, K, nb = 256 * 256, 50, 5
    thr = 112 if iso else 96
    for rec in (0, _lib.MULTI_RECORD):
        small = _lib.multi_workspace_bytes(256, 256, 3, 2, nb, K, fl | rec)      # 30 planes: 2-pass
        with _lib.option("MIN_PLANES", 0):
            fused_small = _lib.multi_workspace_bytes(256, 256, 3, 2, nb, K, fl | rec)
        assert small != fused_small
        planes = 30
        # two spectra of 4 B/px per plane at least, and (recording) the natural s trajectory of 8 B/px per slot
        assert small >= 2 * planes * px * 4 + (49 * planes * px * 8 if rec else 0)
        # the threshold, in planes in all (P * B * nbranch): one plane per image, nbranch = thr below / at it
        below = _lib.multi_workspace_bytes(256, 256, 1, 1, thr - 1, K, fl | rec)
        at = _lib.multi_workspace_bytes(256, 256, 1, 1, thr, K, fl | rec)
        with _lib.option("MIN_PLANES", 0):
            assert _lib.multi_workspace_bytes(256, 256, 1, 1, thr, K, fl | rec) == at
            assert _lib.multi_workspace_bytes(256, 256, 1, 1, thr - 1, K, fl | rec) != below


@pytest.mark.parametrize("case", __import__("paths_table").CASES, ids=[c[0] for c in __import__("paths_table").CASES])
def test_path_decision_table(case):
    """Every (shape, prox, PSF, call, record flags, options) combination takes its intended path: the library's
    one decision table (admm_capi.hip plan_paths) answered through admm_query_paths, host code only.
    tests/test_gpu_paths.py checks on the GPU that these are the kernels that launch."""
    import contextlib
    cid, M, N, iso, kh, mode, flags, hb, rho, opts, fwd, bwd = case
    with contextlib.ExitStack() as st:
        for k, v in opts.items():
            st.enter_context(_lib.option(k, v))
        assert _lib.query_paths(M, N, iso, kh, mode, flags, hb, rho) == (fwd, bwd), cid


@pytest.mark.parametrize("case", __import__("paths_table").PLANE_CASES,
                         ids=[c[0] for c in __import__("paths_table").PLANE_CASES])
def test_path_decision_table_plane_count_rule(case):
    """Small batches go to the 2-pass kernels (ADMM_OPT_MIN_PLANES = -1, the default); 0 switches the rule off and
    a positive value sets one threshold for every per-plane path."""
    cid, M, N, iso, kh, mode, flags, hb, rho, planes, fwd, bwd = case
    assert _lib.get_option("MIN_PLANES") == -1
    assert _lib.query_paths(M, N, iso, kh, mode, flags, hb, rho, planes) == (fwd, bwd), cid
    with _lib.option("MIN_PLANES", 0):
        assert _lib.query_paths(M, N, iso, kh, mode, flags, hb, rho, planes) == \
            _lib.query_paths(M, N, iso, kh, mode, flags, hb, rho, 0), cid
    with _lib.option("MIN_PLANES", planes + 1):
        small = _lib.query_paths(M, N, iso, kh, mode, flags, hb, rho, planes)
        assert small[0] not in ("fused", "fused_iso", "resident", "resident_iso"), cid


def test_query_paths_rejects_negative_planes():
    with pytest.raises(Exception):
        _lib.query_paths(256, 256, False, 0, 0, 0, False, False, -1)
