import sys, os
sys.path[:0] = ['admm-deconv_amd', 'oracle', 'tests']
import numpy as np, torch, admm_deconv
from admm_deconv import synth
h = synth.gaussian_psf(15, 2.5); y = synth.make_batch(2, 256, 256, h, g0=11)
rng = np.random.default_rng(256 + 256 + 25); xbar = rng.standard_normal(y.shape).astype(np.float32)
dev = torch.device('cuda:0')
out = {}
for K in (25, 10, 3):
    x, yb, hb, lb, rb = admm_deconv.tvd_fft_backward(torch.from_numpy(y).to(dev), torch.from_numpy(xbar).to(dev), 0.0041, 0.021, torch.from_numpy(h).to(dev), False, K)
    torch.cuda.synchronize()
    out[f'x{K}'] = x.cpu().numpy(); out[f'yb{K}'] = yb.cpu().numpy(); out[f'hb{K}'] = hb.cpu().numpy(); out[f'lb{K}'] = float(lb); out[f'rb{K}'] = float(rb)
np.savez('gpurun_out/bwd_dump.npz', **out)
print('ok')
