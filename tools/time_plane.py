"""Time the fused per-plane path against the 2-pass path on BASELINE c2 (512 x 256^2, K=25)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "admm-deconv_amd"))
import admm_deconv  # noqa: E402
from admm_deconv import _lib, synth  # noqa: E402

# NAME=VALUE arguments are library options (admm_set_option), e.g. FUSED=0 LINE_T=4 GEN_TM=4096
for _a in [a for a in sys.argv[1:] if "=" in a]:
    _lib.set_option(_a.split("=")[0].upper(), int(_a.split("=")[1]))
    sys.argv.remove(_a)

dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
h = synth.gaussian_psf(15, 2.5)
base = torch.from_numpy(synth.make_batch(64, 256, 256, h)).to(dev)
y = base.repeat((B + 63) // 64, 1, 1, 1)[:B].contiguous()
ht = torch.from_numpy(h).to(dev)
ws = admm_deconv.Workspace()
out = torch.empty_like(y)
for mode in ("1", "0"):
    _lib.set_option("FUSED", int(mode))
    for _ in range(2):
        admm_deconv.tvd_fft(y, 0.0041, 0.021, ht, False, 25, out=out, workspace=ws)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 5
    for _ in range(n):
        admm_deconv.tvd_fft(y, 0.0041, 0.021, ht, False, 25, out=out, workspace=ws)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / n
    _lib.profile_reset()
    _lib.profile_enable(True)
    admm_deconv.tvd_fft(y, 0.0041, 0.021, ht, False, 25, out=out, workspace=ws)
    _lib.profile_enable(False)
    ks = {name: _lib.profile_get(c) for c, name in _lib.KERNEL_CLASSES.items() if _lib.profile_get(c)[1]}
    print(f"fused={mode}: {1000 * el:.3f} ms/solve  {B / el:.0f} img/s  kernels(ms,n)={ks}", flush=True)
