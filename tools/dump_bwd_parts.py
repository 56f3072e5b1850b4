"""Debug: run the GPU backward and dump the per-step (rho_bar, tau_bar) block partials from the workspace."""
import sys
sys.path[:0] = ['admm-deconv_amd', 'oracle', 'tests']
import numpy as np, torch, admm_deconv
from admm_deconv import synth, ops

def align(v): return (v + 255) & ~255
def layout(M, N, planes, kh, kw, K, T, want_h):
    off = 0; L = {}
    def take(name, b):
        nonlocal off; L[name] = off; off = align(off + b)
    MN = M * N
    take('twM', M * 8); take('twN', N * 8); take('C', (M // 2 + 1) * N * 4)
    if kh: take('G', (M // 2 + 1) * N * 8); take('hty', planes * MN * 4)
    take('sA', planes * 2 * MN * 4); take('sB', planes * 2 * MN * 4); take('spec0', planes * MN * 4); take('spec1', planes * MN * 4)
    take('traj_s', max(K - 1, 1) * planes * 2 * MN * 4)
    if want_h and kh: take('traj_v', K * planes * MN * 4); take('sig', (M // 2 + 1) * N * 16)
    take('sbA', planes * 2 * MN * 4); take('sbB', planes * 2 * MN * 4); take('vsum', planes * MN * 4)
    take('rpart', K * planes * (N // T) * 2 * 8)
    return L

M = N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
K = int(sys.argv[2]) if len(sys.argv) > 2 else 3
h = synth.gaussian_psf(15, 2.5); y = synth.make_batch(2, M, N, h, g0=11)
rng = np.random.default_rng(M + N + 25); xbar = rng.standard_normal(y.shape).astype(np.float32)
dev = torch.device('cuda:0')
ws = ops.Workspace()
x, yb, hb, lb, rb = admm_deconv.tvd_fft_backward(torch.from_numpy(y).to(dev), torch.from_numpy(xbar).to(dev), 0.0041, 0.021,
                                                 torch.from_numpy(h).to(dev), False, K, need_h=False, workspace=ws)
torch.cuda.synchronize()
T = 8 if M <= 512 else 4
Lo = layout(M, N, 2, 15, 15, K, T, False)
ptr = ws._buf.data_ptr(); off0 = (-ptr) % 256
raw = ws._buf[off0 + Lo['rpart']: off0 + Lo['rpart'] + K * 2 * (N // T) * 2 * 8].cpu().numpy().view(np.float64)
parts = raw.reshape(K, 2, N // T, 2)   # [K-k][plane][block][rho,tau]
np.savez(f'gpurun_out/bwd_parts_{M}_{K}.npz', parts=parts, lb=float(lb), rb=float(rb), y=y, xbar=xbar)
print('per-step sums (step k=K..1): rho', parts[..., 0].sum(axis=(1, 2)), 'tau', parts[..., 1].sum(axis=(1, 2)))
tr = ws._buf[off0 + Lo['traj_s']: off0 + Lo['traj_s'] + (K - 1) * 2 * 2 * M * N * 4].cpu().numpy().view(np.float32)
np.savez(f'gpurun_out/bwd_traj_{M}_{K}.npz', traj=tr.reshape(K - 1, 2, 2, N, M), x=x.cpu().numpy())
print('traj saved')
