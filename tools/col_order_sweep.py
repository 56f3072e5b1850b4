"""Column plan order sweep for the compile-time-plan kernels (admm_smooth.hip): for every compiled length N,
time the column pass (K = 25 launches) with increasing (ADMM_OPT_SMOOTH = 2) and decreasing (= 3) radices
on 256-pixel lines, ~16 M pixels per solve.  Prints one JSON line per length; the faster order goes into
SM_COL_ASC_LENGTHS.  Usage (GPU box): python tools/col_order_sweep.py [N ...]"""
import json
import os
import re
import sys

import torch

R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(R, "admm-deconv_amd"))
import admm_deconv  # noqa: E402
from admm_deconv import _lib, synth  # noqa: E402

src = open(os.path.join(R, "admm-deconv_amd", "csrc", "admm_smooth.hip")).read()
block = src[src.index("#define SM_LENGTHS(X)"):].split("\n\n")[0]
LENGTHS = [int(v) for v in re.findall(r"X\((\d+)\)", block)]
if len(sys.argv) > 1:
    LENGTHS = [int(a) for a in sys.argv[1:]]


def column_ms(y, h, mode):
    with _lib.option("SMOOTH", mode):
        admm_deconv.tvd_fft(y, synth.LAMBDA, synth.RHO, h, False, 25)
        torch.cuda.synchronize()
        _lib.profile_reset()
        _lib.profile_enable(True)
        admm_deconv.tvd_fft(y, synth.LAMBDA, synth.RHO, h, False, 25)
        _lib.profile_enable(False)
    ms, n = _lib.profile_get(_lib.K_COLUMN)
    return ms


def main():
    dev = torch.device("cuda", 0)
    M = 256
    h = torch.from_numpy(synth.gaussian_psf(5, 1.0)).to(dev)
    for N in LENGTHS:
        B = max(1, (16 << 20) // (M * N))
        y = torch.rand((B, 1, N, M), device=dev)
        a, d = column_ms(y, h, 2), column_ms(y, h, 3)
        print(json.dumps({"N": N, "batch": B, "asc_ms": round(a, 3), "desc_ms": round(d, 3),
                          "best": "asc" if a < 0.97 * d else "desc"}), flush=True)


if __name__ == "__main__":
    main()
