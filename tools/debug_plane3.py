"""Fused path nondeterminism census: mismatching runs vs the 2-pass path for several batch sizes."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "admm-deconv_amd"))
import admm_deconv  # noqa: E402
from admm_deconv import synth  # noqa: E402

dev = torch.device("cuda:0")
K = int(sys.argv[1]) if len(sys.argv) > 1 else 6
for B in (1, 4, 64):
    y = torch.from_numpy(synth.make_batch(min(B, 8), 256, 256, None)).to(dev).repeat((B + 7) // 8, 1, 1, 1)[:B].contiguous()
    os.environ["ADMM_FUSED"] = "0"
    ref = admm_deconv.tvd_fft(y, 0.0041, 0.021, None, False, K)
    os.environ["ADMM_FUSED"] = "1"
    bad_runs, bad_planes = 0, 0
    for _ in range(10):
        a = admm_deconv.tvd_fft(y, 0.0041, 0.021, None, False, K)
        e = ((a - ref).flatten(1).norm(dim=1) / ref.flatten(1).norm(dim=1)).cpu().numpy()
        nb = int((e > 1e-5).sum())
        bad_planes += nb
        bad_runs += nb > 0
    print(f"B={B} K={K}: runs with a bad plane {bad_runs}/10, bad planes {bad_planes}/{10 * B}", flush=True)
