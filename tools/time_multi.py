"""Time the c5 one-grid multi-branch forward (recording ST masks) and reverse sweep of a given library build
(experiments: tools/build_variant.sh makes libadmm_deconv_<TAG>.so).  usage: time_multi.py [TAG ...]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "admm-deconv_amd"))
from admm_deconv import _lib, synth  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else ""
if tag:
    _lib.LIB_PATH = os.path.join(REPO, "admm-deconv_amd", f"libadmm_deconv_{tag}.so")
import admm_deconv  # noqa: E402

dev = torch.device("cuda", 0)
B, P, K = int(os.environ.get("B", 64)), 3, int(os.environ.get("K", 50))
y = torch.from_numpy(synth.make_batch(8, 256, 256, None, P=P, sigma=0.1)).to(dev).repeat(B // 8, 1, 1, 1)
lams = [torch.tensor([0.004 * (i + 1)], device=dev) for i in range(5)]
rhos = [torch.tensor([r], device=dev) for r in (0.002, 0.02, 0.2, 2.0, 4.0)]
xb = torch.randn((B, 5 * P, 256, 256), device=dev)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
tf, ta = [], []
for it in range(4):
    ev[0].record()
    x, rec = admm_deconv.tvd_fft_multi(y, lams, rhos, K, record=True, need_rho=False)
    ev[1].record()
    admm_deconv.tvd_fft_multi_backward_recorded(rec, x, xb, need_y=False, need_rho=False)
    ev[2].record()
    torch.cuda.synchronize()
    if it:
        tf.append(ev[0].elapsed_time(ev[1]))
        ta.append(ev[1].elapsed_time(ev[2]))
print(f"{tag or 'base'}: forward {min(tf):.3f} ms  adjoint {min(ta):.3f} ms  ({5 * B * P} planes, K={K})", flush=True)
