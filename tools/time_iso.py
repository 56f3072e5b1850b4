"""Time the isotropic 256 x 256 forward: split-iteration per-plane kernels (default) against the 2-pass path
(option FUSED = 0).  usage: time_iso.py [planes] [K]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "admm-deconv_amd"))
import admm_deconv  # noqa: E402
from admm_deconv import _lib, synth  # noqa: E402

dev = torch.device("cuda", 0)
planes = int(sys.argv[1]) if len(sys.argv) > 1 else 192
K = int(sys.argv[2]) if len(sys.argv) > 2 else 50
y = torch.from_numpy(synth.make_batch(16, 256, 256, None, P=1, sigma=0.1)).to(dev).repeat(planes // 16, 1, 1, 1)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
out = {}
for fused in (1, 0):
    with _lib.option("FUSED", fused):
        ts = []
        for it in range(4):
            ev[0].record()
            x = admm_deconv.tvd_fft(y, 0.0041, 0.2, None, True, K)
            ev[1].record()
            torch.cuda.synchronize()
            if it:
                ts.append(ev[0].elapsed_time(ev[1]))
        out[fused] = (min(ts), x)
d = (out[1][1] - out[0][1]).abs().max().item() / out[0][1].abs().max().item()
print(f"iso {planes} planes K={K}: split-iteration {out[1][0]:.3f} ms, 2-pass {out[0][0]:.3f} ms, max rel diff {d:.2e}",
      flush=True)

# the adjoint: recorded without rho_bar (the fused sweep) against the 2-pass sweep (option FUSED_ADJ = 0)
xb = torch.randn_like(y)
res = {}
for fa in (1, 0):
    with _lib.option("FUSED_ADJ", fa):
        tr, tb = [], []
        for it in range(4):
            ev[0].record()
            x, rec = admm_deconv.tvd_fft_record(y, 0.0041, 0.2, None, True, K, need_rho=False)
            ev[1].record()
            torch.cuda.synchronize()
            e2 = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            e2[0].record()
            yb, _, lb, _ = admm_deconv.tvd_fft_backward_recorded(rec, x, xb, need_rho=False)
            e2[1].record()
            torch.cuda.synchronize()
            if it:
                tr.append(ev[0].elapsed_time(ev[1]))
                tb.append(e2[0].elapsed_time(e2[1]))
        res[fa] = (min(tr), min(tb), yb, float(lb))
d = (res[1][2] - res[0][2]).norm().item() / res[0][2].norm().item()
print(f"iso adjoint {planes} planes K={K}: fused record {res[1][0]:.3f} + sweep {res[1][1]:.3f} ms, "
      f"2-pass record {res[0][0]:.3f} + sweep {res[0][1]:.3f} ms; y_bar rel L2 diff {d:.2e}, "
      f"lambda_bar {res[1][3]:.6e} vs {res[0][3]:.6e}", flush=True)
