"""Debug aid: the fused forward's ST mask-byte trajectory (ADMM_REC_MASKS) against masks formed from a full
s_k recording of the same solve (lane-native layouts, read back through libadmm_devtest.so's offsets)."""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "admm-deconv_amd"), os.path.join(REPO, "tests"), os.path.join(REPO, "oracle")]
import admm_deconv  # noqa: E402
from admm_deconv import synth  # noqa: E402

dev = torch.device("cuda", 0)
K, B = 4, 1
y = torch.from_numpy(synth.make_batch(B, 256, 256, None, P=1, sigma=0.1, g0=3)).to(dev)
lam, rho = 0.05, 0.2
tau = np.float32(np.float32(lam) / np.float32(rho))


def raw(rec, nbytes):
    buf = rec.workspace._buf
    ptr, _ = rec.workspace.get(0, buf.device)
    base = ptr - buf.data_ptr()
    lib = ctypes.CDLL(os.path.join(REPO, "admm-deconv_amd", "libadmm_devtest.so"))
    ts, tn = ctypes.c_size_t(0), ctypes.c_size_t(0)
    lib.devtest_recording_offsets.argtypes = [ctypes.c_int] * 8 + [ctypes.POINTER(ctypes.c_size_t)] * 2
    lib.devtest_recording_offsets(256, 256, 1, B, 0, K, 0, 0, ctypes.byref(ts), ctypes.byref(tn))
    return buf[base + ts.value: base + ts.value + nbytes].cpu().numpy()


x1, r1 = admm_deconv.tvd_fft_record(y, lam, rho, None, False, K, need_h=False)
torch.cuda.synchronize()
s = raw(r1, (K - 1) * B * 64 * 512 * 16).view(np.float32).reshape(K - 1, B, 64, 512, 4)
x2, r2 = admm_deconv.tvd_fft_record(y, lam, rho, None, False, K, need_h=False, need_rho=False)
torch.cuda.synchronize()
m = raw(r2, (K - 1) * B * 16 * 512 * 4).view(np.uint32).reshape(K - 1, B, 16, 512)
print("x equal:", bool(torch.equal(x1, x2)))
# expected bytes from s
mb = (np.abs(s) > tau).astype(np.uint32)
sg = (s.view(np.uint32) >> 31).astype(np.uint32)
byte = mb[..., 0] | mb[..., 1] << 1 | mb[..., 2] << 2 | mb[..., 3] << 3 | (sg[..., 0] | sg[..., 1] << 1 | sg[..., 2] << 2 | sg[..., 3] << 3) << 4
exp = np.zeros((K - 1, B, 16, 512), np.uint32)
for n in range(64):
    exp[:, :, n >> 2] |= byte[:, :, n] << (8 * (n & 3))
for k in range(K - 1):
    d = exp[k] != m[k]
    print(f"slot {k}: mismatching dwords {int(d.sum())} of {d.size}; mask bits set expected {int(mb[k].sum())}")
    if d.any():
        idx = np.argwhere(d)[:5]
        for i in idx:
            print("   at", tuple(i), hex(int(exp[k][tuple(i)])), hex(int(m[k][tuple(i)])))
xb = torch.randn_like(y)
a = admm_deconv.tvd_fft_backward_recorded(r1, x1, xb)
b = admm_deconv.tvd_fft_backward_recorded(r2, x2, xb, need_rho=False)
torch.cuda.synchronize()
print("lambda_bar full", float(a[2]), "masks", float(b[2]), "y_bar equal", bool(torch.equal(a[0], b[0])))
