"""Does splitting one batch over several HIP streams (each part its own workspace, launched back to back) fill the
kernel-boundary tails of the 2-pass path?  Times the whole batch as one call against S parts on S streams.

usage (GPU box): python tools/stream_split_probe.py [--config c4] [--splits 1 2 3 4] [--steps 5]
One JSON line per split count: ms per step (the whole batch solved) and img/s.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "admm-deconv_amd"))

import torch  # noqa: E402

import admm_deconv  # noqa: E402
from admm_deconv import synth  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--splits", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=0)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = dict(synth.CONFIGS[a.config])
    B = a.batch or cfg["B"]
    y, h, _, _ = bench.make_inputs(cfg, B, 0, 64, dev)
    out = torch.empty_like(y)
    K = cfg["K"]
    for S in a.splits:
        parts = [(y[i * B // S:(i + 1) * B // S], out[i * B // S:(i + 1) * B // S]) for i in range(S)]
        streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(S - 1)]
        ws = [admm_deconv.Workspace() for _ in range(S)]
        main_s = streams[0]

        def step():
            for s in streams[1:]:
                s.wait_stream(main_s)
            for (yp, xp), s, w in zip(parts, streams, ws):
                admm_deconv.tvd_fft(yp, synth.LAMBDA, synth.RHO, h, False, K, out=xp, workspace=w, stream=s)
            for s in streams[1:]:
                main_s.wait_stream(s)

        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        print(json.dumps({"config": a.config, "batch": B, "splits": S, "ms_per_step": round(1000 * el / a.steps, 3),
                          "img_s": round(B * a.steps / el, 1)}), flush=True)


if __name__ == "__main__":
    main()
