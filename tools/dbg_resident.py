import os, sys, json
import numpy as np, torch
sys.path.insert(0, "admm-deconv_amd"); sys.path.insert(0, "oracle")
import admm_deconv, oracle_np
from admm_deconv import _lib, synth
dev = torch.device("cuda", 0)
M = N = 250
hp = synth.gaussian_psf(15, 2.5)
out = {}
for K in (1, 2):
    for with_h in (False, True):
        yb = synth.make_batch(1, M, N, hp if with_h else None)
        y = torch.from_numpy(yb).to(dev)
        hh = torch.from_numpy(hp).to(dev) if with_h else None
        with _lib.option("RESIDENT", 1):
            a = admm_deconv.tvd_fft(y, synth.LAMBDA, synth.RHO, hh, False, K).cpu().numpy()[0, 0]
        with _lib.option("RESIDENT", 0):
            b = admm_deconv.tvd_fft(y, synth.LAMBDA, synth.RHO, hh, False, K).cpu().numpy()[0, 0]
        d = np.abs(a - b)
        rows = d.max(axis=1); cols = d.max(axis=0)
        key = f"K{K}_h{int(with_h)}"
        out[key] = {"rel": float(np.linalg.norm(a - b) / np.linalg.norm(b)),
                    "bad_rows": np.nonzero(rows > 1e-3 * np.abs(b).max())[0][:40].tolist(),
                    "n_bad_rows": int((rows > 1e-3 * np.abs(b).max()).sum()),
                    "bad_cols": np.nonzero(cols > 1e-3 * np.abs(b).max())[0][:40].tolist(),
                    "n_bad_cols": int((cols > 1e-3 * np.abs(b).max()).sum()),
                    "ratio_mean": float((a * b).sum() / (b * b).sum()),
                    "a00": a[:3, :3].tolist(), "b00": b[:3, :3].tolist()}
        print(key, json.dumps(out[key]), flush=True)
        np.save(f"gpurun_out/dbg_{key}_a.npy", a); np.save(f"gpurun_out/dbg_{key}_b.npy", b)
