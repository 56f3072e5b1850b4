"""Fused path: run-to-run determinism and the first K at which it departs from the 2-pass path."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "admm-deconv_amd"))
import admm_deconv  # noqa: E402
from admm_deconv import synth  # noqa: E402

dev = torch.device("cuda:0")
y = torch.from_numpy(synth.make_batch(4, 256, 256, None)).to(dev)
for K in (3, 4, 5, 6, 8):
    os.environ["ADMM_FUSED"] = "1"
    runs = [admm_deconv.tvd_fft(y, 0.0041, 0.021, None, False, K).cpu().numpy().astype(np.float64) for _ in range(3)]
    os.environ["ADMM_FUSED"] = "0"
    b = admm_deconv.tvd_fft(y, 0.0041, 0.021, None, False, K).cpu().numpy().astype(np.float64)
    det = [float(np.abs(r - runs[0]).max()) for r in runs[1:]]
    errs = [float(np.linalg.norm(runs[0][i] - b[i]) / np.linalg.norm(b[i])) for i in range(4)]
    d = np.abs(runs[0][0, 0] - b[0, 0])
    loc = np.argwhere(d > 1e-4)
    print(f"K={K} run-to-run maxdiff={det} rel per plane={['%.1e' % e for e in errs]} n_bad={len(loc)} "
          f"first={loc[:6].tolist()}")
