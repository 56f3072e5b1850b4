"""Solve time against the number of planes, path against path (measurement tool, not part of the product).

  python tools/time_small.py [--iso] [--bwd] SIDE OPT=A/B PLANES...
  e.g. python tools/time_small.py 256 FUSED=1/0 1 2 8 32 64 96 128 192

For every plane count the forward (tvd_fft; with --bwd the recording forward plus its reverse sweep, y_bar
and lam_bar wanted) runs with the library option at value A and at value B, K = 25 (--bwd: K = 50), 15 x 15
Gaussian PSF; one JSON line per point with the planned path (admm_query_paths) and the time per call from
CUDA events over 20 calls.  Used to place the small-batch rules of plan_paths."""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "admm-deconv_amd"))
import admm_deconv  # noqa: E402
from admm_deconv import _lib, synth  # noqa: E402


def main():
    argv = sys.argv[1:]
    iso = "--iso" in argv
    bwd = "--bwd" in argv
    argv = [a for a in argv if not a.startswith("--")]
    side = int(argv[0])
    name, vals = argv[1].split("=")
    va, vb = (int(v) for v in vals.split("/"))
    planes = [int(p) for p in argv[2:]]
    K = 50 if bwd else 25
    dev = torch.device("cuda", 0)
    hp = synth.gaussian_psf(15, 2.5)
    h = torch.from_numpy(hp).to(dev)
    base = torch.from_numpy(synth.make_batch(8, side, side, hp)).to(dev)
    lam = torch.tensor([synth.LAMBDA], device=dev)
    rho = torch.tensor([synth.RHO], device=dev)

    def call(y):
        if not bwd:
            return admm_deconv.tvd_fft(y, lam, rho, h, iso, K)
        x, rec = admm_deconv.ops.tvd_fft_record(y, lam, rho, h, iso, K, need_h=False, need_rho=False)
        return admm_deconv.ops.tvd_fft_backward_recorded(rec, x, torch.ones_like(x), need_y=True, need_rho=False)

    for n in planes:
        y = base.repeat((n + 7) // 8, 1, 1, 1)[:n].contiguous()
        row = {"side": side, "planes": n, "iso": iso, "bwd": bwd, "K": K}
        for v in (va, vb):
            with _lib.option(name, v):
                mode = _lib.MODE_RECORD if bwd else _lib.MODE_FORWARD
                paths = _lib.query_paths(side, side, iso, 15, mode, _lib.REC_MASKS if bwd else 0)
                for _ in range(3):
                    call(y)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    call(y)
                e1.record()
                torch.cuda.synchronize()
            row[f"{name}={v}"] = {"path": paths[0], "ms": round(e0.elapsed_time(e1) / 20, 4)}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
