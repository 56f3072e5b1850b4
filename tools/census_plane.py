"""Fused-path census: bad planes vs the 2-pass path and run-to-run equality, PSF and no-PSF, full c2
batch.  Prints one line per case; any nonzero count is a failure."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "admm-deconv_amd"))
import admm_deconv  # noqa: E402
from admm_deconv import _lib, synth  # noqa: E402

dev = torch.device("cuda:0")
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 5
tot_bad = 0
for psf in (True, False):
    h = synth.gaussian_psf(15, 2.5) if psf else None
    ht = None if h is None else torch.from_numpy(h).to(dev)
    y = torch.from_numpy(synth.make_batch(64, 256, 256, h)).to(dev).repeat(8, 1, 1, 1).contiguous()
    for K in (3, 8):
        _lib.set_option("FUSED", int("0"))
        ref = admm_deconv.tvd_fft(y, 0.0041, 0.021, ht, False, K)
        _lib.set_option("FUSED", int("1"))
        first = None
        bad_ref = bad_rr = 0
        for _ in range(runs):
            a = admm_deconv.tvd_fft(y, 0.0041, 0.021, ht, False, K)
            e = (a - ref).flatten(1).norm(dim=1) / ref.flatten(1).norm(dim=1)
            bad_ref += int((e > 1e-5).sum())
            if first is None:
                first = a
            else:
                bad_rr += int((a != first).flatten(1).any(dim=1).sum())
        tot_bad += bad_ref + bad_rr
        print(f"psf={psf} K={K}: planes checked {runs * 512}, bad vs 2-pass {bad_ref}, run-to-run mismatching {bad_rr}",
              flush=True)
print("CENSUS", "PASS" if tot_bad == 0 else "FAIL", tot_bad)
