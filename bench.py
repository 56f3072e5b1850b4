"""Benchmark: ADMM TV-deconvolution images/s at 256x256, K=25 (BASELINE.json metric, config c2).

One "step" = one full tvd_fft solve (src/ops/ops.jl:181 semantics) of a batch of synthetic
Gaussian-blurred 256x256 images (15x15 PSF, lambda 0.0041, rho 0.021, K = 25, anisotropic) that is
already resident in HBM, through the HIP library's C ABI.

  N = 1 (default): BASELINE c2, batch 512 on one GPU.
  N > 1: BASELINE c3, batch 2048 sharded over the N GPUs (2048/N images per GPU, one process per GPU,
         RCCL over xGMI) plus the RCCL gather of every output to rank 0 inside the timed region.  The
         gather of one batch runs on its own stream and overlaps the solve of the next
         (admm_deconv.parallel.ShardGather).  `python bench.py --gpus N` spawns the N ranks itself; the
         driver's `torchrun --nproc-per-node N bench.py --gpus N` sets RANK/WORLD_SIZE and is used as is.

Prints ONE JSON line on rank 0.  Besides the driver's keys it carries
  roofline      -- dominant kernel: algorithmic bytes per launch / measured avg launch duration
                   (hipEvents on the launch stream, via the library profiler) vs 8 TB/s HBM peak;
                   `traffic` = PMC-measured HBM bytes per launch from profiles/ when available.
  cpu_baseline  -- the C restatement of the reference CPU solve (oracle/admm_oracle.c, fp32, OpenMP)
                   timed on this host on a bounded sample of the same workload (rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "admm-deconv_amd"))
# c5 runs its 5 Parallel branches on 5 HIP streams (layers.Parallel); HIP maps streams onto
# GPU_MAX_HW_QUEUES hardware queues (4 by default), and streams sharing a queue serialise.  Must be set
# before the HIP runtime initialises (c5: 1.50k -> 1.60k img/s with 8).
if "c5" in sys.argv:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import admm_deconv  # noqa: E402
from admm_deconv import _lib, parallel, synth  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X spec (MI355X_MICROARCH.md, chip-level parameters)


def achievable_gbs():
    """The best rate a hand-written gfx950 stream of the solve kernels' own 12:8 read/write mix reaches
    (tools/ubench/stream.hip, profiles/r05_hbm_ceiling.json), or None."""
    try:
        d = json.load(open(os.path.join(REPO, "profiles", "r05_hbm_ceiling.json")))
        return 1000.0 * float(d["achievable_mixed_TBps"])
    except Exception:   # noqa: BLE001
        return None


def canonical_bytes(M, N, K):
    """per plane K*[32*(M/2+1)*N + 20*M*N] + 12*M*N."""
    return K * (32 * (M // 2 + 1) * N + 20 * M * N) + 12 * M * N


def plane_bytes_per_px(K):
    """Fused per-plane kernel (plane_kernel.hip), HBM bytes per pixel for one K-iteration solve:
    y in (4) + H^T y out (4) + (K-1) x H^T y in (4) + (K-2) x [s out (8) + s in (8)] + x out (4)
    (s_k is written for k = 1..K-2 and read by the next iteration; s_{K-1} is never read).
    The line spectrum never leaves the CU, so this is the algorithm's minimum."""
    return 12 + 4 * (K - 1) + 16 * max(K - 2, 0)


def kernel_bytes_per_plane(M, N, K):
    """Algorithmic bytes per plane for one launch of each kernel class (SURVEY.md s8d split)."""
    H = M // 2 + 1
    return {
        "column": 16 * H * N,                 # read + write the half spectrum
        "line": 16 * H * N + 20 * M * N,      # spectrum in/out + s in/out (2 ch) + H^T y
        "prep": 8 * M * N + 8 * H * N,        # y in, H^T y out, spectrum out
        "final": 8 * H * N + 4 * M * N,       # spectrum in, x out
        "plane": plane_bytes_per_px(K) * M * N,   # whole fused solve
    }


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one process per GPU); spawned here unless "
                    "launched by torchrun")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default=None, choices=sorted(synth.CONFIGS),
                    help="default: c2 on one GPU, c3 (2048 global, sharded + gathered) on N > 1")
    ap.add_argument("--batch", type=int, default=None, help="images per GPU (default: the config's; c3 -> 2048/N)")
    ap.add_argument("--no-gather", action="store_true", help="N > 1: skip the gather to rank 0 (solve only)")
    ap.add_argument("--chunks", type=int, default=1, help="N > 1: slices per shard, each gathered as soon as solved")
    ap.add_argument("--gather-engine", default="both", choices=("both", "ipc", "rccl"),
                    help="N > 1: 'ipc' = every rank copies its solved slices into rank 0's IPC-shared receive buffer "
                         "(async peer copies, SDMA: no CU held); 'rccl' = dist.gather over RCCL (falls back to it "
                         "when the IPC handle cannot be opened); 'both' (default) = the metric with ipc, plus the "
                         "same steps with rccl timed in the same invocation (per-rank diagnostics)")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="N > 1: nccl (RCCL over xGMI); gloo only to rehearse the schedule with ranks sharing a GPU")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="library option (admm_set_option), e.g. FUSED=0 or LINE_T=4; experiments only")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample duration")
    ap.add_argument("--distinct", type=int, default=64, help="distinct synthetic images generated per rank (tiled)")
    ap.add_argument("--serial-branches", action="store_true",
                    help="c5: run the Parallel branches one after the other on one stream (the reference's order)")
    ap.add_argument("--no-merge", action="store_true",
                    help="c5: solve the Parallel branches one by one (per-branch streams) instead of one grid")
    ap.add_argument("--merge-iso", action="store_true",
                    help="c5 --iso: the branches in one grid (ADMM_MULTI_ISO) at any batch (default: only when all their planes fit one wave of workgroups, layers.ISO_MERGE_MAX_PLANES)")
    ap.add_argument("--iso", action="store_true",
                    help="c5 only: isotropic (BT) prox in the layers (use_iso, src/configs/train_cfg.json:14)")
    ap.add_argument("--graph", dest="graph", action="store_true", default=None,
                    help="c5: capture the whole training step (forward, loss, adjoint, update) in one HIP graph and "
                         "replay it.  Default: on when the merged branches run the 2-pass kernels (below the "
                         "library's plane-count rule: the reference's train_cfg.json batch 2), whose ~400 launches "
                         "per step make the step launch-bound (profiles/r05_c5_small_batch_graph.jsonl); off above")
    ap.add_argument("--no-graph", dest="graph", action="store_false")
    return ap.parse_args()


def make_inputs(cfg, B, g0, distinct, dev):
    psf = synth.gaussian_psf(*cfg["psf"]) if cfg["psf"] else None
    nd = min(B, distinct)
    base = synth.make_batch(nd, cfg["M"], cfg["N"], psf, P=cfg["P"], g0=g0)
    reps = (B + nd - 1) // nd
    y = np.concatenate([base] * reps)[:B]
    return (torch.from_numpy(np.ascontiguousarray(y)).to(dev), None if psf is None else torch.from_numpy(psf).to(dev),
            psf, base)


def iso_fused_bytes_per_px(K):
    """HBM bytes per pixel of one isotropic solve's plane256_iso_kernel launches (all K) and plane256_isoadj_kernel
    launches (all K; no y_bar, no rho_bar: the c5 layers' case) -- DESIGN.md s3.
    Forward: k = 0 y in, H^T y out, s_1 out, q out (4 + 4 + 8 + 4); 0 < k < K-1: H^T y, s_k (B phase), s_k
    again, s_{k+1}, q (A phase) (4 + 8 + 8 + 8 + 4); k = K-1: H^T y, s_k, x out (4 + 8 + 4).
    Reverse step k: B phase (k < K) vbar_{k+1} in, s_k in, sbar_{k+1} in (k + 1 < K), sbar_k out (4 + 8 + 8 + 8);
    k = K: x_bar in (4); A phase (k >= 2) vbar_k out, s_{k-1} in, sbar_k in (k < K), R partial out (4 + 8 + 8 + 4)."""
    if K == 1:
        return 8.0, 4.0
    fwd = 20 + 32 * (K - 2) + 16
    adj = 0
    for k in range(K, 0, -1):
        adj += 4 if k == K else 4 + 8 + (8 if k + 1 < K else 0) + 8
        if k >= 2:
            adj += 4 + 8 + (8 if k < K else 0) + 4
    return float(fwd), float(adj)


def bench_c5(args, dev):
    """BASELINE c5: the denoiser branch of src/nets/net_build.jl:113-128 (5 x ADMMDeconvF2((), 50, rho, relu1)
    in Parallel(chcat)), batch 64 of 256x256 RGB; one step = forward + GMSD loss + backward through the HIP
    adjoint + SGD update of the trainable lambda (the layers' trainable set, deconv_admm.jl:107)."""
    from admm_deconv import layers, metrics
    cfg = synth.CONFIGS["c5"]
    M, N, P, B, K = cfg["M"], cfg["N"], cfg["P"], args.batch or cfg["B"], cfg["K"]
    rng = np.random.default_rng(0)
    branch = [layers.ADMMDeconvF2((), K, r, layers.relu1, iso=args.iso, rng=rng, device=dev)
              for r in (0.002, 0.02, 0.2, 2.0, 4.0)]
    for L in branch:
        L.lam.requires_grad_(True)
    nd = min(B, args.distinct)
    noisy = synth.make_batch(nd, M, N, None, P=P, sigma=0.1)
    clean = synth.make_clean(nd, M, N, P=P)
    reps = (B + nd - 1) // nd
    x = torch.from_numpy(np.concatenate([noisy] * reps)[:B]).to(dev)
    target = torch.from_numpy(np.concatenate([clean] * reps)[:B]).to(dev).repeat(1, len(branch), 1, 1)

    net = layers.Parallel(layers.chcat, *branch, streams=not args.serial_branches,   # net_build.jl:121-125
                          merge=False if (args.no_merge or args.serial_branches) else ("always" if args.merge_iso else True))
    merged = net._mergeable(x)

    def step():
        out = net(x)                                          # 5 branches on their own HIP streams, chcat
        loss = metrics.gmsd_loss(out, target)                 # the training loss, src/train.jl:129,191
        loss.backward()
        with torch.no_grad():
            for L in branch:
                L.lam -= 1e-3 * L.lam.grad
                L.lam.grad = None
        return loss

    run = step
    graph = None
    if args.graph is None:
        # the merged grid below the plane-count rule (ADMM_OPT_MIN_PLANES default; 96 aniso / 112 iso planes in
        # all) runs the 2-pass kernels: ~100 launches per direction and branch set, so one graph per step pays
        # (c5 batch 2: iso 401 -> 418, aniso 578 -> 617 img/s on one box); above it the step is one launch per
        # solve (aniso) or per iteration on per-branch streams (iso), where a graph gains nothing or loses
        args.graph = bool(merged and _lib.get_option("MIN_PLANES") == -1 and
                          len(branch) * B * P < (112 if args.iso else 96))
    if args.graph:
        # warm up on a side stream (allocations, recordings registry, kernel attributes), then capture one whole
        # step; replays re-run every kernel of it (the gradients are recomputed, not accumulated: grad is None
        # going into the capture, so backward() writes fresh tensors from the graph's pool)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(max(args.warmup, 2)):
                step()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step()
        run = graph.replay
    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    # per-kernel timing from a separate instrumented step with the branches serialised, so that each
    # launch's hipEvent duration is its own (concurrent branches share the CUs)
    net.use_streams = False
    _lib.profile_reset()
    _lib.profile_enable(True)
    step()
    _lib.profile_enable(False)
    net.use_streams = not args.serial_branches
    kernels = {}
    for cls, name in _lib.KERNEL_CLASSES.items():
        ms, n = _lib.profile_get(cls)
        if n:
            kernels[name] = {"launches_per_step": n, "avg_ms": ms / n, "total_ms_per_step": ms}
    roof = None
    planes = B * P
    if merged and "column" in kernels:
        # below the plane-count rule (the reference's training batch of 2: 30 planes) the merged grid runs the
        # 2-pass kernels over all branches' planes (admm_launch.hip run_multi_2pass_*).  Algorithmic bytes per
        # pixel of a launch, per class (the per-branch f / |s| / R maps are L2-resident, not counted):
        #   column  packed line spectrum in + out                                           8
        #   iso     line    iso_a: spectrum 4, s_k 8, s_k+1 8 | iso_b: s 8, H^T y 4, spectrum 4    (20 + 16) / 2
        #           adjoint iso_adj_a: spectrum 4, s_k-1 8, sbar 8, vbar 4, Vsum 8 | iso_adj_b: vbar 4, sbar 8,
        #                   s_k-1 8, sbar out 8, spectrum 4                                        (32 + 32) / 2
        #   aniso   line    spectrum in 4 + out 4, s_k-1 8, s_k 8, H^T y 4                              28
        #           adjoint line_adj: spectrum in 4 + out 4, s_k-1 8, sbar in 8 + out 8 (no rho_bar, no y_bar)  32
        nb = len(branch)
        px = nb * planes * M * N
        per = {"column": 8 * px, "line": (18 if args.iso else 28) * px, "adjoint": 32 * px}
        for k, b in per.items():
            if k in kernels:
                kernels[k]["algorithmic_bytes_per_launch"] = b
                kernels[k]["achieved_GBps"] = round(b / (kernels[k]["avg_ms"] * 1e-3) / 1e9, 1)
        dom = max((k for k in per if k in kernels), key=lambda k: kernels[k]["total_ms_per_step"])
        a = kernels[dom]
        ach = per[dom] / (a["avg_ms"] * 1e-3) / 1e9
        roof = {"bound": "hbm", "kernel": f"{dom} (2-pass {'isotropic ' if args.iso else ''}kernels, one grid of {nb} "
                                          f"branches x {planes} planes)",
                "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                "traffic": load_traffic("c5iso2m", dom, planes=nb * planes) if args.iso else None,
                "algorithmic_bytes_per_launch": per[dom], "avg_launch_ms": round(a["avg_ms"], 5)}
    elif merged and args.iso:
        # one grid of 5 x 192 planes per iteration / reverse step (plane_iso.hip, ADMM_MULTI_ISO)
        fwd, adj = iso_fused_bytes_per_px(K)
        nb = len(branch)
        per = {"plane": nb * planes * M * N * fwd / K, "adjoint": nb * planes * M * N * adj / K}
        for k, b in per.items():
            if k in kernels:
                kernels[k]["algorithmic_bytes_per_launch"] = b
                kernels[k]["achieved_GBps"] = round(b / (kernels[k]["avg_ms"] * 1e-3) / 1e9, 1)
        dom = max((k for k in per if k in kernels), key=lambda k: kernels[k]["total_ms_per_step"])
        a = kernels[dom]
        ach = per[dom] / (a["avg_ms"] * 1e-3) / 1e9
        roof = {"bound": "hbm", "kernel": f"{dom} (plane_iso.hip, one grid of {nb} branches x {planes} planes, "
                                          f"{K} launches)", "achieved": round(ach, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                "traffic": load_traffic("c5isom", dom, planes=nb * planes), "algorithmic_bytes_per_launch": per[dom],
                "avg_launch_ms": round(a["avg_ms"], 5)}
    elif merged:
        # one grid of 5 x 192 planes for the forward (plane256_kernel recording ST mask bits: lambda is the
        # only trainable, rho_bar is not formed) and one for the reverse sweep (plane256_adj_kernel<masks>).
        # Per pixel: forward y in, H^T y copy out (4 + 4), per iteration H^T y in (4, K-1 times), s in / out
        # (8 + 8, K-2 times), mask byte per pixel pair out (0.5, K-1 times), x out (4);
        # reverse: x_bar in (4), per step sbar in, sbar out (8 + 8), mask in (0.5), K-1 times each
        nb = len(branch)
        fwd_px = 12 + 4 * (K - 1) + 16 * (K - 2) + 0.5 * (K - 1)
        adj_px = 4 + 16.5 * (K - 1)
        per = {"plane": nb * planes * M * N * fwd_px, "adjoint": nb * planes * M * N * adj_px}
        for k, b in per.items():
            if k in kernels:
                kernels[k]["algorithmic_bytes_per_launch"] = b
                kernels[k]["achieved_GBps"] = round(b / (kernels[k]["avg_ms"] * 1e-3) / 1e9, 1)
        dom = max((k for k in per if k in kernels), key=lambda k: kernels[k]["total_ms_per_step"])
        a = kernels[dom]
        ach = per[dom] / (a["avg_ms"] * 1e-3) / 1e9
        roof = {"bound": "hbm", "kernel": f"{dom} (one grid of {nb} branches x {planes} planes)", "achieved": round(ach, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                "traffic": load_traffic("c5m", dom, planes=nb * planes), "algorithmic_bytes_per_launch": per[dom],
                "avg_launch_ms": round(a["avg_ms"], 5)}
    elif args.iso and kernels.get("plane", {}).get("launches_per_step") == len(branch) * K:
        # isotropic at 256 x 256: the split-iteration kernels of plane_iso.hip, one plane256_iso_kernel per
        # iteration and one plane256_isoadj_kernel per reverse step (the batch norm / R sums between them are
        # "norm").  Per pixel of a launch (the branch's 256 KiB f / R / |s| maps are L2-resident, not counted):
        fwd, adj = iso_fused_bytes_per_px(K)
        nb = len(branch)
        per = {"plane": planes * M * N * fwd / K, "adjoint": planes * M * N * adj / K}
        for k, b in per.items():
            if k in kernels:
                kernels[k]["algorithmic_bytes_per_launch"] = b
                kernels[k]["achieved_GBps"] = round(b / (kernels[k]["avg_ms"] * 1e-3) / 1e9, 1)
        dom = max((k for k in per if k in kernels), key=lambda k: kernels[k]["total_ms_per_step"])
        a = kernels[dom]
        ach = per[dom] / (a["avg_ms"] * 1e-3) / 1e9
        roof = {"bound": "hbm", "kernel": f"{dom} (plane_iso.hip, {nb} branches x {K} launches)", "achieved": round(ach, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                "traffic": load_traffic("c5iso", dom, planes=planes), "algorithmic_bytes_per_launch": per[dom],
                "avg_launch_ms": round(a["avg_ms"], 5)}
    elif not args.iso and kernels.get("adjoint", {}).get("launches_per_step") == len(branch):
        # fused reverse sweep (plane256_adj_kernel, one launch per layer).  The input and rho need no gradient,
        # so the sweep gets neither y_bar nor rho_bar and reads no Vsum and no s_k; per pixel: the ST mask
        # byte of s_{k-1} (one byte per lane pixel pair: 0.5 B/px), sbar_k in, sbar_{k-1} out (K-1 steps each, 8 B)
        # and x_bar in (4 B): 4 + 16.5 (K - 1) B/px
        per_launch = planes * M * N * (4 + 16.5 * (K - 1))
        a = kernels["adjoint"]
        ach = per_launch / (a["avg_ms"] * 1e-3) / 1e9
        roof = {"bound": "hbm", "kernel": "adjoint (plane256_adj)", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": load_traffic("c5", "adjoint", planes=planes),
                "algorithmic_bytes_per_launch": per_launch, "avg_launch_ms": round(a["avg_ms"], 5)}
    elif not args.iso and "adjoint" in kernels:
        # line_adj per plane and reverse step: packed line spectrum in + out (8 (M/2) N each), s_{k-1},
        # sbar_k, sbar_{k-1} (8 M N each; no s_k and no Vsum: neither rho_bar nor y_bar requested)
        per_launch = planes * (16 * (M // 2) * N + 24 * M * N)
        a = kernels["adjoint"]
        ach = per_launch / (a["avg_ms"] * 1e-3) / 1e9
        roof = {"bound": "hbm", "kernel": "adjoint (line_adj)", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                "algorithmic_bytes_per_launch": per_launch, "avg_launch_ms": round(a["avg_ms"], 5)}
    print(json.dumps({
        "metric": "c5 ADMM denoiser-branch train step (fwd + adjoint) images/s", "value": round(B * args.steps / el, 2),
        "unit": "images/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1000 * el / args.steps, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": f"c5: batch {B} of {M}x{N}x{P}, 5 x ADMMDeconvF2((), {K}, rho, relu1) + chcat, "
                               "GMSD loss (HIP), backward through the recorded adjoint "
                               f"({'iso' if args.iso else 'aniso'}; "
                               f"{'branches in one grid' if merged else 'per-branch solves'}"
                               f"{'; whole step replayed as one HIP graph' if graph is not None else ''})",
                   "global_batch": B},
        "roofline": roof, "kernels": kernels}))


def cpu_baseline(cfg, psf, base, target_s):
    """Time the C restatement (fp32, OpenMP) on a bounded sample of the same workload."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_c
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    n = max(1, min(threads, base.shape[0]))
    sample = np.ascontiguousarray(base[:n])
    t0 = time.perf_counter()
    done = 0
    runs = 0
    while True:
        oracle_c.tvd_fft_c(sample, synth.LAMBDA, synth.RHO, psf, False, cfg["K"], np.float32, nthreads=threads)
        done += n
        runs += 1
        el = time.perf_counter() - t0
        if el >= target_s or runs >= 2000:
            break
    return {
        "value": done / el, "unit": "images/s", "cores": threads, "kind": "port",
        "sample": f"{runs} x {n} images of {cfg['M']}x{cfg['N']}x{cfg['P']}, K={cfg['K']}, "
                  f"{cfg['psf'][0]}x{cfg['psf'][0]} PSF, {el:.1f} s wall; C restatement of ops.jl:17-96 "
                  f"(oracle/admm_oracle.c, fp32, OpenMP over planes)",
    }


def load_traffic(cfg_name, kernel, key="hbm_bytes_per_launch", planes=None):
    """A PMC figure per launch from profiles/pmc_traffic.json, or None.  The profiled launch's plane count is
    recorded with it ("planes"): a launch over another number of planes gets None, not the profiled bytes (a
    committed profile describes the launch it measured, not this one)."""
    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        e = d.get(cfg_name, {}).get(kernel)
        if e is None or (planes is not None and e.get("planes") != planes):
            return None
        return e.get(key)
    except Exception:
        return None


# VALU issue peak: 4 SIMDs per CU, each issuing a wave64 fp32 VALU instruction every 2 cycles
# (MI355X_MICROARCH.md, per-instruction constants), 256 CUs, 2.4 GHz
VALU_ISSUE_PEAK = 256 * 2 * 2.4e9   # wave-instructions per second


def compute_side(cfg_name, kernel, avg_ms, planes):
    """Compute-side figure of the dominant kernel: SQ_INSTS_VALU per launch (PMC, profiles/pmc_traffic.json)
    over the chip's VALU issue peak for the measured launch time (None off the profiled plane count)."""
    valu = load_traffic(cfg_name, kernel, "valu_insts_per_launch", planes)
    if not valu:
        return None
    rate = valu / (avg_ms * 1e-3)
    return {"valu_insts_per_launch": valu, "valu_issue_rate": rate, "valu_issue_peak": VALU_ISSUE_PEAK,
            "valu_issue_frac": round(rate / VALU_ISSUE_PEAK, 4),
            "lds_insts_per_launch": load_traffic(cfg_name, kernel, "lds_insts_per_launch", planes),
            "wait_any_frac": load_traffic(cfg_name, kernel, "wait_any_frac", planes)}


def spawn_ranks(n):
    """`python bench.py --gpus N` without torchrun: start N rank processes (one per GPU) before this
    process touches the GPU, and exit with the worst of their exit codes.  Only rank 0 prints."""
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    sys.exit(bad[0] if bad else 0)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if "WORLD_SIZE" in os.environ and args.gpus not in (1, world):
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    for kv in args.opt:
        k, v = kv.split("=")
        _lib.set_option(k.strip().upper(), int(v))
    config = args.config or ("c2" if world == 1 else "c3")
    if config == "c5":
        return bench_c5(args, torch.device("cuda", 0))
    if world > 1:
        if args.backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local if args.backend == "nccl" else local % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    cfg = dict(synth.CONFIGS[config])
    if args.batch:
        B = args.batch
    elif config == "c3":
        B = cfg["B"] // world
    else:
        B = cfg["B"]
    M, N, P, K = cfg["M"], cfg["N"], cfg["P"], cfg["K"]
    gather = world > 1 and not args.no_gather
    y, h, psf_np, base = make_inputs(cfg, B, g0=rank * B, distinct=args.distinct, dev=dev)
    out = torch.empty_like(y)
    ws = [admm_deconv.Workspace() for _ in range(max(1, args.chunks))]
    stream = torch.cuda.current_stream(dev)
    chunk_of = {}

    def solve(ys, xs):
        # one workspace per chunk slot (chunks of one step are enqueued back to back on one stream)
        i = chunk_of.setdefault(ys.data_ptr(), len(chunk_of) % len(ws))
        admm_deconv.tvd_fft(ys, synth.LAMBDA, synth.RHO, h, False, K, out=xs, workspace=ws[i], stream=stream)

    engine = "ipc" if args.gather_engine == "both" else args.gather_engine
    # stream_only: nothing reads the gathered batches between steps (ShardGather's ipc rule)
    sg = parallel.ShardGather(y, solve, chunks=args.chunks, engine=engine, stream_only=True) if gather else None

    def step():
        if sg is not None:
            sg.step()
        else:
            solve(y, out)

    def timed(body, steps, sg=sg):
        """Barrier + synchronize on both sides of `steps` calls of body; (this rank's seconds, max over ranks,
        ms from this rank's last solve being enqueued to the end of its device work)."""
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            body()
        solved = torch.cuda.Event(enable_timing=True)
        solved.record(stream)                # after the last solve on the compute stream
        if sg is not None:
            sg.wait()                        # the compute stream waits for this rank's gathers / peer copies
        done = torch.cuda.Event(enable_timing=True)
        done.record(stream)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        mx = el
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev if args.backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            mx = float(t.item())
        return el, mx, solved.elapsed_time(done)

    for _ in range(args.warmup):
        step()
    el_rank, el, tail_ms = timed(step, args.steps)
    images = B * world * args.steps
    value = images / el
    ms_per_step = 1000.0 * el / max(args.steps, 1)

    ranks = None
    solve_only = None
    if world > 1:
        # diagnostics for the multi-GPU record (outside the timed region above): the same steps solve-only (no
        # gather) in this invocation, and per rank what it saw -- which engine ran, how long its own steps took,
        # how long its gathers ran past its last solve, and which device it drove
        so_rank, so_el, _ = timed(lambda: solve(y, out), args.steps) if gather else (el_rank, el, 0.0)
        # the other gather engine on the same shards and steps (--gather-engine both): the first multi-GPU
        # record then compares the IPC push with the RCCL gather
        alt = None
        if gather and args.gather_engine == "both":
            # a diagnostic leg: an error in it is reported in the record instead of losing the metric above
            other = "rccl" if sg.engine == "ipc" else "ipc"
            try:
                sg2 = parallel.ShardGather(y, solve, chunks=args.chunks, engine=other, stream_only=True)
                for _ in range(args.warmup):
                    sg2.step()
                a_rank, a_el, a_tail = timed(sg2.step, args.steps, sg=sg2)
                alt = {"engine": sg2.engine, "ms_per_step": round(1000.0 * a_rank / args.steps, 4),
                       "max_ms_per_step": round(1000.0 * a_el / args.steps, 4), "value": round(images / a_el, 2),
                       "gather_tail_ms": round(a_tail, 4)}
                sg2.close()
            except Exception as e:   # noqa: BLE001
                alt = {"engine": other, "error": repr(e)[:300]}
        props = torch.cuda.get_device_properties(dev)
        me = {"rank": rank, "world_seen": dist.get_world_size(), "backend": dist.get_backend(),
              "device": dev.index, "visible_devices": torch.cuda.device_count(),
              "device_uuid": str(getattr(props, "uuid", "")), "pci_bus_id": getattr(props, "pci_bus_id", None),
              "gather_engine": (sg.engine if sg is not None else None),
              "ms_per_step": round(1000.0 * el_rank / args.steps, 4),
              "solve_only_ms_per_step": round(1000.0 * so_rank / args.steps, 4),
              "gather_tail_ms": round(tail_ms, 4),
              "other_engine": alt}
        ranks = [None] * world
        dist.all_gather_object(ranks, me)
        solve_only = {"ms_per_step": round(1000.0 * so_el / args.steps, 4),
                      "value": round(images / so_el, 2),
                      "note": "same steps and shards without the gather, max over ranks (not the metric)"}
        if alt is not None and "error" not in alt:
            solve_only["other_engine"] = {"engine": alt["engine"], "ms_per_step": alt["max_ms_per_step"],
                                          "value": alt["value"],
                                          "note": "same steps gathered by the other engine, max over ranks (not the metric)"}

    # ---- per-kernel timing (separate instrumented solve; not part of the timed region) ----
    _lib.profile_reset()
    _lib.profile_enable(True)
    reps = 2
    for _ in range(reps):
        admm_deconv.tvd_fft(y, synth.LAMBDA, synth.RHO, h, False, K, out=out, workspace=ws[0], stream=stream)
    _lib.profile_enable(False)
    planes = B * P
    # planes per launch: the MALL-resident schedule runs large 2-pass batches as chunks on several streams
    chunk, nstreams = _lib.forward_schedule(M, N, False, cfg["psf"][0], planes)
    kb = kernel_bytes_per_plane(M, N, K)
    kernels = {}
    for cls, name in _lib.KERNEL_CLASSES.items():
        ms, n = _lib.profile_get(cls)
        if n == 0:
            continue
        avg_ms = ms / n
        e = {"launches_per_solve": n // reps, "avg_ms": avg_ms, "total_ms_per_solve": ms / reps}
        if name in kb:
            e["algorithmic_bytes_per_launch"] = kb[name] * chunk
            e["achieved_GBps"] = kb[name] * chunk / (avg_ms * 1e-3) / 1e9
        kernels[name] = e
    dom = max((k for k in kernels if k in kb), key=lambda k: kernels[k]["total_ms_per_solve"])
    alg_bytes = kb["plane"] * planes if "plane" in kernels else canonical_bytes(M, N, K) * planes
    traffic = load_traffic(config, dom, planes=chunk)
    ach = kernels[dom]["achieved_GBps"]
    roofline = {
        "bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
        # against the measured streaming ceiling of the same read/write mix (not the 8 TB/s spec)
        "achievable_peak": achievable_gbs(),
        "frac_of_achievable": round(ach / achievable_gbs(), 4) if achievable_gbs() else None,
        "algorithmic_bytes_per_launch": kernels[dom]["algorithmic_bytes_per_launch"],
        "avg_launch_ms": round(kernels[dom]["avg_ms"], 5),
        "compute": compute_side(config, dom, kernels[dom]["avg_ms"], chunk),
        # launches of `chunk_planes` planes; with streams > 1 that many chunks' launches run concurrently, so a
        # launch's duration includes its share of the chip (the whole-solve figure below is the aggregate)
        # (rocprofv3's begin -> end of the same launches is shorter: profiles/r06_c4_mall_kernel_stats.csv, DESIGN.md
        # s5); overlap = the kernels' event time per solve over the solve's wall time
        "schedule": {"chunk_planes": chunk, "streams": nstreams,
                     "overlap": round(sum(k["total_ms_per_solve"] for k in kernels.values()) / ms_per_step, 2)},
        # with streams > 1: the dominant class's algorithmic bytes per solve over its share of the solve's wall time
        # (its share of the summed event time) -- an estimate of the rate the concurrent launches reach together
        "concurrent_estimate": None if nstreams <= 1 else {
            "achieved_GBps": round(kernels[dom]["algorithmic_bytes_per_launch"] * kernels[dom]["launches_per_solve"]
                                   / (ms_per_step * 1e-3 * kernels[dom]["total_ms_per_solve"]
                                      / sum(k["total_ms_per_solve"] for k in kernels.values())) / 1e9, 1)},
        "whole_solve": {
            # the bytes of the path that ran (fused: plane_bytes_per_px; 2-pass: SURVEY s8d canonical)
            "algorithmic_bytes": alg_bytes,
            "achieved_GBps": round(alg_bytes / (ms_per_step * 1e-3) / 1e9, 1),
            "frac": round(alg_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            # SURVEY.md s8d's byte model of the 2-pass form (the spectrum round-trips through HBM twice per
            # iteration): what a 2-pass solve would have to move, NOT bytes this run moved
            "survey_2pass_model_bytes": canonical_bytes(M, N, K) * planes,
        },
    }

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, psf_np, base, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "ADMM deconv images/sec at 256x256 K=25 (% HBM roofline)",
            "value": round(value, 2), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            # c3 fixes the global batch (2048 split over the ranks): strong scaling; c2/c4 fix the per-GPU batch
            "scaling": "strong" if (config == "c3" and not args.batch) else "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"{config}: batch {B}/GPU of {M}x{N}x{P}, {cfg['psf'][0]}x{cfg['psf'][0]} "
                                   f"Gaussian PSF (sigma {cfg['psf'][1]}), K={K}, anisotropic TV, lambda {synth.LAMBDA}, "
                                   f"rho {synth.RHO}", "global_batch": B * world, "image": [M, N, P], "K": K,
                       "parallelism": f"batch-shard x{world}" + (
                           (" + IPC push gather (async peer copies over xGMI)" if sg.engine == "ipc" else
                            " + RCCL gather" if args.backend == "nccl" else " + gloo gather") + " (overlapped, "
                           f"{args.chunks} chunk{'s' if args.chunks > 1 else ''}/shard)" if gather else "")},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "kernels": kernels,
        }
        if ranks is not None:
            line["ranks"] = ranks
            line["solve_only"] = solve_only
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
