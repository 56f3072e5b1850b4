"""Localise fused-vs-2-pass differences (debug aid): per K, error magnitude by line and pixel."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "admm-deconv_amd"))
import admm_deconv  # noqa: E402
from admm_deconv import synth  # noqa: E402

dev = torch.device("cuda:0")
for psf in (True, False):
    h = synth.gaussian_psf(15, 2.5) if psf else None
    y = torch.from_numpy(synth.make_batch(1, 256, 256, h)).to(dev)
    ht = None if h is None else torch.from_numpy(h).to(dev)
    for K in (1, 2, 3, 5):
        os.environ["ADMM_FUSED"] = "1"
        a = admm_deconv.tvd_fft(y, 0.0041, 0.021, ht, False, K)[0, 0].cpu().numpy().astype(np.float64)
        os.environ["ADMM_FUSED"] = "0"
        b = admm_deconv.tvd_fft(y, 0.0041, 0.021, ht, False, K)[0, 0].cpu().numpy().astype(np.float64)
        d = np.abs(a - b)
        rel = np.linalg.norm(a - b) / np.linalg.norm(b)
        rows = d.max(axis=1)   # per line j
        cols = d.max(axis=0)   # per pixel i
        bad_r = np.where(rows > 1e-3 * np.abs(b).max())[0]
        bad_c = np.where(cols > 1e-3 * np.abs(b).max())[0]
        print(f"psf={psf} K={K} rel={rel:.3e} max={d.max():.3e} |b|max={np.abs(b).max():.3e} "
              f"bad lines({len(bad_r)}): {bad_r[:20].tolist()} bad px({len(bad_c)}): {bad_c[:20].tolist()}")
        if K == 2 and len(bad_r):
            j = bad_r[0]
            print("   line", j, "a:", np.round(a[j, :8], 5).tolist(), "b:", np.round(b[j, :8], 5).tolist())
