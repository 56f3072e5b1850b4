"""Small-batch isotropic 256 x 256 solve + reverse sweep: the per-plane fused kernels against the 2-pass
kernels at a few plane counts (the batch-2 training step has 30 planes on 256 CUs).

usage (GPU box): python tools/small_batch_probe.py [--planes 6,30,60] [--iters 10]
One JSON line per (planes, path): ms per record-forward and per reverse sweep (K = 50, HIP events).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "admm-deconv_amd"))

import torch  # noqa: E402

from admm_deconv import _lib, ops  # noqa: E402


def run(planes, path, iters, K, iso):
    torch.manual_seed(0)
    y = torch.rand(planes, 1, 256, 256, device="cuda")
    xb = torch.randn_like(y)
    lam = torch.full((1,), 0.02, device="cuda")
    rho = torch.full((1,), 0.3, device="cuda")
    _lib.set_option("MIN_PLANES", 0 if path == "fused" else 1 << 20)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tf = tb = 0.0
    for i in range(iters + 2):
        ev[0].record()
        x, rec = ops.tvd_fft_record(y, lam, rho, None, iso, K, need_h=False, need_rho=False)
        ev[1].record()
        ops.tvd_fft_backward_recorded(rec, x, xb, need_y=True, need_rho=False)
        ev[2].record()
        torch.cuda.synchronize()
        if i >= 2:
            tf += ev[0].elapsed_time(ev[1])
            tb += ev[1].elapsed_time(ev[2])
    _lib.set_option("MIN_PLANES", -1)
    return tf / iters, tb / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--planes", default="6,30,60")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--K", type=int, default=50)
    ap.add_argument("--aniso", action="store_true")
    a = ap.parse_args()
    for p in [int(v) for v in a.planes.split(",")]:
        for path in ("fused", "2pass"):
            f, b = run(p, path, a.iters, a.K, not a.aniso)
            print(json.dumps({"planes": p, "path": path, "iso": not a.aniso, "K": a.K, "fwd_ms": round(f, 3),
                              "bwd_ms": round(b, 3), "per_iter_us": round(1e3 * (f + b) / a.K, 1)}), flush=True)


if __name__ == "__main__":
    main()
