"""Is the c4 MALL-resident schedule host-bound?  Times the host enqueue of one c4 solve (the call's return) against
the solve's completion, and the GPU time from events.  GPU box only.  usage: python tools/c4_enqueue_probe.py"""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "admm-deconv_amd"))
import admm_deconv  # noqa: E402
from admm_deconv import _lib, synth  # noqa: E402


def main():
    cfg = synth.CONFIGS["c4"]
    M, N, P, K = cfg["M"], cfg["N"], cfg["P"], cfg["K"]
    dev = torch.device("cuda", 0)
    base = synth.make_batch(16, M, N, synth.gaussian_psf(*cfg["psf"]), P=P)
    y = torch.from_numpy(np.concatenate([base] * 16)).to(dev)
    h = torch.from_numpy(synth.gaussian_psf(*cfg["psf"])).to(dev)
    out = torch.empty_like(y)
    ws = admm_deconv.Workspace()
    for n in (4, 1):
        _lib.set_option("MALL_STREAMS", n)
        for _ in range(2):
            admm_deconv.tvd_fft(y, synth.LAMBDA, synth.RHO, h, False, K, out=out, workspace=ws)
        torch.cuda.synchronize()
        rows = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record()
            admm_deconv.tvd_fft(y, synth.LAMBDA, synth.RHO, h, False, K, out=out, workspace=ws)
            t1 = time.perf_counter()
            e1.record()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            rows.append((1e3 * (t1 - t0), 1e3 * (t2 - t0), e0.elapsed_time(e1)))
        print(json.dumps({"mall_streams": n, "schedule": _lib.forward_schedule(M, N, False, 15, y.shape[0] * P),
                          "enqueue_ms": [round(r[0], 2) for r in rows], "wall_ms": [round(r[1], 2) for r in rows],
                          "event_ms": [round(r[2], 2) for r in rows]}), flush=True)
    _lib.set_option("MALL_STREAMS", 4)


if __name__ == "__main__":
    main()
