"""GPU: the kernels that actually launch for every combination of tests/paths_table.py are those of the path the
library's decision table (admm_capi.hip plan_paths, queried by admm_query_paths) names.  Counted through the
library profiler's kernel classes (include/admm_deconv.h ADMM_K_*), K = 4 iterations:
  forward  fused / resident: one ADMM_K_PLANE launch; fused_iso / resident_iso: K (one per iteration); 2-pass, smooth and
           runtime-length paths: none (column / line kernels instead);
  sweep    sweep_fused: one ADMM_K_ADJ launch; sweep_fused_iso: K and no column pass anywhere in the call;
           2-pass and runtime-length sweeps: >= K - 1 adjoint launches and column passes."""
import contextlib

import numpy as np
import pytest
import torch

import admm_deconv
from admm_deconv import _lib, synth
from paths_table import CASES, HBAR, MASKS, PLANE_CASES

pytestmark = pytest.mark.gpu
K = 4


def _counts():
    return {name: _lib.profile_get(cls)[1] for cls, name in _lib.KERNEL_CLASSES.items()}


def _run_and_check(dev, cid, M, N, iso, kh, mode, flags, hb, rho, planes, fwd, bwd):
    h = synth.gaussian_psf(kh, 1.0) if kh else None
    ht = None if h is None else torch.from_numpy(h).to(dev)
    y = torch.from_numpy(synth.make_batch(planes, M, N, h)).to(dev)
    xb = torch.randn_like(y)
    assert _lib.query_paths(M, N, iso, kh, mode, flags, hb, rho, planes) == (fwd, bwd), cid
    _lib.profile_reset()
    _lib.profile_enable(True)
    try:
        if mode == 0:
            admm_deconv.tvd_fft(y, 0.0041, 0.021, ht, iso, K)
        elif mode == 1:
            x, rec = admm_deconv.tvd_fft_record(y, 0.0041, 0.021, ht, iso, K, need_h=bool(flags & HBAR),
                                                need_rho=not flags & MASKS)
            admm_deconv.tvd_fft_backward_recorded(rec, x, xb, need_rho=not flags & MASKS)
        else:
            admm_deconv.tvd_fft_backward(y, xb, 0.0041, 0.021, ht, iso, K, need_h=hb, need_rho=rho)
        torch.cuda.synchronize()
    finally:
        _lib.profile_enable(False)
    c = _counts()
    plane, adj, col = c.get("plane", 0), c.get("adjoint", 0), c.get("column", 0)
    want_plane = {"fused": 1, "resident": 1, "fused_iso": K, "resident_iso": K}.get(fwd, 0)
    assert plane == want_plane, f"{cid}: forward path {fwd} but {plane} plane launches ({c})"
    if bwd == "sweep_fused":
        assert adj == 1, f"{cid}: {c}"
    elif bwd == "sweep_fused_iso":
        assert adj == K and col == 0, f"{cid}: {c}"
    elif bwd is not None:
        assert adj >= K - 1 and col > 0, f"{cid}: {c}"
    if fwd not in ("fused", "resident", "fused_iso", "resident_iso"):
        assert col >= K, f"{cid}: {c}"


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_launched_kernels_follow_the_decision_table(dev, case):
    """2 planes, the plane-count rule off (conftest), options as the table gives them."""
    cid, M, N, iso, kh, mode, flags, hb, rho, opts, fwd, bwd = case
    with contextlib.ExitStack() as st:
        for k, v in opts.items():
            st.enter_context(_lib.option(k, v))
        _run_and_check(dev, cid, M, N, iso, kh, mode, flags, hb, rho, 2, fwd, bwd)


@pytest.mark.min_planes_rule
@pytest.mark.parametrize("case", PLANE_CASES, ids=[c[0] for c in PLANE_CASES])
def test_launched_kernels_follow_the_plane_count_rule(dev, case):
    """The library's defaults: below the measured plane counts the 2-pass kernels run (ADMM_OPT_MIN_PLANES = -1)."""
    cid, M, N, iso, kh, mode, flags, hb, rho, planes, fwd, bwd = case
    assert _lib.get_option("MIN_PLANES") == -1
    _run_and_check(dev, cid, M, N, iso, kh, mode, flags, hb, rho, planes, fwd, bwd)
