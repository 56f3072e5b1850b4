"""c4 (512^2 x 3, batch 256, K = 50) solved in plane chunks whose per-iteration working set fits the Infinity
Cache (VERDICT r05 Next #3), against the whole batch in one call.  GPU box only.

A 2-pass iteration touches, per 512^2 plane: the packed spectrum twice (column in / out, line in / out: 2 x 1 MiB),
s in and out (2 x 2 MiB) and H^T y (1 MiB) -- about 7 MiB; 24 planes are ~170 MiB, inside the 256 MiB MALL.  Each
chunk runs all K iterations before the next starts.  Variants: one stream, chunks back to back; and two streams
taking alternate chunks (each kernel's tail overlaps the other stream's next kernel; two chunks' sets in cache).

usage: python tools/c4_chunk_probe.py [--chunks 16,24,32,48,64] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "admm-deconv_amd"))
import admm_deconv  # noqa: E402
from admm_deconv import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", default="16,24,32,48,64")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--streams", default="1,2")
    a = ap.parse_args()
    cfg = synth.CONFIGS["c4"]
    M, N, P, K = cfg["M"], cfg["N"], cfg["P"], cfg["K"]
    dev = torch.device("cuda", 0)
    nd = 16
    base = synth.make_batch(nd, M, N, synth.gaussian_psf(*cfg["psf"]), P=P)
    y = torch.from_numpy(np.concatenate([base] * (a.batch // nd))).to(dev).reshape(-1, 1, N, M)   # planes
    h = torch.from_numpy(synth.gaussian_psf(*cfg["psf"])).to(dev)
    planes = y.shape[0]
    out = torch.empty_like(y)
    nsmax = max(int(v) for v in a.streams.split(","))
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(device=dev) for _ in range(nsmax - 1)]
    ws = [admm_deconv.Workspace() for _ in streams]

    def solve(c, nstreams):
        if c >= planes:
            admm_deconv.tvd_fft(y, synth.LAMBDA, synth.RHO, h, False, K, out=out, workspace=ws[0], stream=streams[0])
            return
        for k in range(1, nstreams):
            streams[k].wait_stream(streams[0])
        for i, p0 in enumerate(range(0, planes, c)):
            si = i % nstreams
            admm_deconv.tvd_fft(y[p0:p0 + c], synth.LAMBDA, synth.RHO, h, False, K, out=out[p0:p0 + c],
                                workspace=ws[si], stream=streams[si])
        for k in range(1, nstreams):
            streams[0].wait_stream(streams[k])

    solve(planes, 1)
    torch.cuda.synchronize()
    ref = out.clone()
    variants = [(planes, 1)] + [(int(c), int(ns)) for c in a.chunks.split(",") for ns in a.streams.split(",")]
    for c, ns in variants:
        solve(c, ns)   # warm-up (workspace sizes, kernel attributes)
        torch.cuda.synchronize()
        same = bool(torch.equal(out, ref))
        ts = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            solve(c, ns)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ms = 1e3 * min(ts)
        print(json.dumps({"chunk_planes": min(c, planes), "streams": ns, "ms_best": round(ms, 3),
                          "ms_all": [round(1e3 * t, 3) for t in ts], "images_per_s": round(a.batch / (ms * 1e-3), 1),
                          "working_set_MiB": round(min(c, planes) * 7 * ns, 1), "bitwise_whole_batch": same}),
              flush=True)


if __name__ == "__main__":
    main()
