"""GPU: the isotropic prox over a batch sharded across 2 processes sharing the one GPU (gloo carries
the M x N maps through admm_batch_reducer; on a multi-GPU node the same call runs over RCCL).
The shards must reassemble the single-process solve of the whole batch (forward and adjoint), up to
the fp32 rounding of the differently ordered batch sums.  64^2 runs the 2-pass kernels; 256^2 the
split-iteration kernels of plane_iso.hip (their batch sums split into shard sum / all-reduce / factor),
with the fused reverse sweep when rho_bar is not requested."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import admm_deconv
from admm_deconv import parallel, synth

pytestmark = pytest.mark.gpu

B, K = 6, 8
LAM, RHO = 0.0041, 0.021


def _inputs(M, nb=B):
    h = synth.gaussian_psf(7, 1.2)
    y = synth.make_batch(nb, M, M, h)
    xbar = np.random.default_rng(11).standard_normal(y.shape).astype(np.float32)
    return h, y, xbar


def _lane_native(M, need_rho):
    """Whether the isotropic recording keeps s / |s| lane-native (the fused 256^2 sweep, recorded without rho_bar;
    with rho_bar the PSF's h_bar trajectory takes the 2-pass layout) -- test_gpu_adjoint_masked.run_case's rule."""
    from admm_deconv import _lib
    return M == 256 and not need_rho and _lib.get_option("FUSED") == 1 and _lib.get_option("FUSED_ADJ") == 1


def _record_and_replay(y, xbar, h, need_rho, dev, group=None):
    """Forward recorded (sharded with `group`), its batch norms |s_1..s_{K-1}| read back, then the replay:
    (x, |s_k| maps (K-1, M, M), y_bar, h_bar, lam_bar, rho_bar) as host values."""
    import test_gpu_adjoint_masked as tm
    yt, xt, ht = (torch.from_numpy(a).to(dev) for a in (y, xbar, h))
    x, rec = admm_deconv.tvd_fft_record(yt, LAM, RHO, ht, True, K, need_h=need_rho, need_rho=need_rho, group=group)
    torch.cuda.synchronize()
    _, nrm = tm.read_trajectory(rec, K, _lane_native(y.shape[-1], need_rho))
    yb, hb, lb, rb = admm_deconv.tvd_fft_backward_recorded(rec, x, xt, need_rho=need_rho)
    torch.cuda.synchronize()
    return (x.cpu().numpy(), np.array(nrm), yb.cpu().numpy(), None if hb is None else hb.cpu().numpy(), float(lb),
            None if rb is None else float(rb))


def _worker(rank, world, port, q, M, need_rho, resident=0, nb=B, min_planes=0):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from admm_deconv import _lib
    _lib.set_option("RESIDENT", resident if resident else 1)
    # 0: the parent's reference solve runs the per-plane kernels too (conftest); > 0: a threshold the shards
    # straddle (a sharded isotropic call must ignore it)
    _lib.set_option("MIN_PLANES", min_planes)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    h, y, xbar = _inputs(M, nb)
    start, count = parallel.shard_range(nb, world, rank)
    dev = torch.device("cuda", 0)
    ys = torch.from_numpy(y[start:start + count]).to(dev)
    xb = torch.from_numpy(xbar[start:start + count]).to(dev)
    ht = torch.from_numpy(h).to(dev)
    g = dist.group.WORLD
    x = admm_deconv.tvd_fft(ys, LAM, RHO, ht, True, K, group=g)
    x2, yb, hb, lb, rb = admm_deconv.tvd_fft_backward(ys, xb, LAM, RHO, ht, True, K, group=g, need_h=need_rho,
                                                      need_rho=need_rho)
    torch.cuda.synchronize()
    rec = _record_and_replay(y[start:start + count], xbar[start:start + count], h, need_rho, dev, group=g)
    q.put((rank, x.cpu().numpy(), x2.cpu().numpy(), yb.cpu().numpy(), None if hb is None else hb.cpu().numpy(),
           float(lb), None if rb is None else float(rb), rec))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rel(a, b):
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / np.linalg.norm(b))


@pytest.mark.parametrize("M,need_rho,resident", [(64, True, 0), (256, True, 0), (256, False, 0), (120, False, 2)],
                         ids=["2pass", "fused-fwd", "fused-fwd+sweep", "resident-iso"])
def test_iso_sharded_two_processes(dev, M, need_rho, resident):
    """resident-iso: 120 x 120 with ADMM_OPT_RESIDENT = 2, the isotropic CU-resident solve (resident_iso_kernel),
    whose norm kernel splits into the shard sum, the reducer and the factor the same way."""
    from admm_deconv import _lib
    _lib.set_option("RESIDENT", resident if resident else 1)
    try:
        _iso_sharded(dev, M, need_rho, resident)
    finally:
        _lib.set_option("RESIDENT", 1)


@pytest.mark.parametrize("rule", [4, 0], ids=["rule4", "norule"])
@pytest.mark.parametrize("need_rho", [False, True], ids=["sweep", "rho"])
def test_iso_uneven_shards_straddling_the_plane_count_rule(dev, need_rho, rule):
    """7 planes at 256^2 on 2 ranks are shards of 4 and 3.  With ADMM_OPT_MIN_PLANES = 4 a shard's
    own plane count would put rank 0 on the fused isotropic kernels and rank 1 on the 2-pass ones, which hand
    the reducer their sum maps in different layouts.  A sharded call ignores the rule, so both take the
    per-plane kernels and the shards reassemble the single-process solve."""
    from admm_deconv import _lib
    assert parallel.shard_range(7, 2, 0)[1] == 4 and parallel.shard_range(7, 2, 1)[1] == 3
    _lib.set_option("MIN_PLANES", 4)
    try:
        assert _lib.query_paths(256, 256, True, 7, planes=4)[0] == "fused_iso"
        assert _lib.query_paths(256, 256, True, 7, planes=3)[0] == "2pass_iso"
    finally:
        _lib.set_option("MIN_PLANES", 0)
    _iso_sharded(dev, 256, need_rho, 0, nb=7, min_planes=rule)


def _iso_sharded(dev, M, need_rho, resident, nb=B, min_planes=0):
    """The sharded solve against the fp64 oracle conditioned on ITS OWN trajectory's BT branches (the shards'
    common batch norms), with the bounds of test_gpu_adjoint_masked.py (<= 1e-5, or the fp32 evaluation's error of
    the same computation); the single-process solve the same way; and every BT branch in which the two runs
    differ lies within rounding of tau in both (the sharded batch norm sums the planes in another order).  That
    is the whole difference between them: the shards compute the exact adjoint of their own trajectory."""
    import test_gpu_adjoint_masked as tm
    import oracle_torch
    if resident:
        from admm_deconv import _lib
        assert _lib.query_paths(M, M, True, 7)[0] == "resident_iso"
    h, y, xbar = _inputs(M, nb)
    ht = torch.from_numpy(h).to(dev)
    x0 = admm_deconv.tvd_fft(torch.from_numpy(y).to(dev), LAM, RHO, ht, True, K).cpu().numpy()
    single = _record_and_replay(y, xbar, h, need_rho, dev)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, M, need_rho, resident, nb, min_planes))
             for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    x = np.concatenate([r[1] for r in res])
    assert _rel(x, x0) < 1e-5
    assert _rel(np.concatenate([r[2] for r in res]), x0) < 1e-5
    # the recorded sharded solve: both ranks hold the same batch norms (the reducer's all-reduced maps)
    recs = [r[7] for r in res]
    assert np.array_equal(recs[0][1], recs[1][1])
    xs = np.concatenate([r[0] for r in recs])
    ybs = np.concatenate([r[2] for r in recs])
    hbs = None if recs[0][3] is None else sum(r[3] for r in recs)   # shard contributions add up
    lbs = sum(r[4] for r in recs)
    rbs = None if recs[0][5] is None else sum(r[5] for r in recs)
    tau = np.float32(np.float32(LAM) / np.float32(RHO))
    masks = oracle_torch.masks_from_trajectory(None, LAM, RHO, True, recs[0][1])
    frac = tm.assert_prox_active(tm.mask_fraction(masks), f"sharded-{M}", False)
    cid = f"sharded-iso-{M}-{nb}planes-{'rho' if need_rho else 'sweep'}"
    err, ref32 = tm.compare_to_oracle(cid, y, xbar, h, LAM, RHO, K, True, masks, frac, xs, ybs, hbs, lbs, rbs)
    # the single-process recording, the same way
    masks1 = oracle_torch.masks_from_trajectory(None, LAM, RHO, True, single[1])
    err1, ref1 = tm.compare_to_oracle(cid + "-single", y, xbar, h, LAM, RHO, K, True, masks1, tm.mask_fraction(masks1),
                                      *single[:1], *single[2:])
    n1, ns = np.asarray(single[1], np.float64), np.asarray(recs[0][1], np.float64)
    flip = (n1 > tau) != (ns > tau)
    diag = (f"flips {int(flip.sum())}, |nrm_single - nrm_sharded| max {np.abs(n1 - ns).max():.3e} "
            f"(rel {np.abs(n1 - ns).max() / np.abs(n1).max():.2e}); single vs its oracle {err1}; "
            f"sharded y_bar vs single {_rel(ybs, single[2]):.3e}, x {_rel(xs, single[0]):.3e}; combined-call sharded "
            f"y_bar vs single {_rel(np.concatenate([r[3] for r in res]), single[2]):.3e}, per rank rec vs comb "
            f"{[_rel(r[7][2], r[3]) for r in res]}")
    print(cid, diag, flush=True)
    # the unsharded solve against its own branches: test_gpu_adjoint_masked.py's bound (<= 1e-5, or the fp32
    # evaluation's error of the same computation)
    tm.check(cid + "-single", err1, ref1)
    # the sharded solve against its own branches: the same bound, or -- sharding must add no error of its own --
    # the unsharded solve's error on the same computation (+5 % for the shards' reordered fp32 batch sums).  The
    # 256^2 sweep cases run the fused isotropic kernels, whose H^T y still passes every iteration's fp32 transforms
    # and sits at the fp32 level; the 2-pass paths are an order of magnitude below it.
    for k in err:
        bound = max(tm.TOL, ref32.get(k, 0.0), 1.05 * err1.get(k, 0.0))
        assert err[k] <= bound, f"{cid}: {k} error {err[k]:.3e} > {bound:.3e} (gpu {err}, fp32 {ref32}); {diag}"
    # the two runs side by side: where no BT branch differs, only the shards' summation order separates them
    if not flip.any():
        assert _rel(ybs, single[2]) <= 2e-5, diag
    # where the two runs' BT branches differ, both norms are within rounding of tau
    if flip.any():
        dist_tau = np.maximum(np.abs(n1[flip] - tau), np.abs(ns[flip] - tau)) / tau
        assert dist_tau.max() <= 1e-4, f"{int(flip.sum())} branch flips, up to {dist_tau.max():.2e} of tau away"
