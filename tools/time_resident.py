"""CU-resident smooth-size solve (admm_resident.hip) against the 2-pass smooth kernels (ADMM_OPT_RESIDENT = 0)
and the numpy oracle: rel-L2 on small batches, then images/s and per-kernel ms at the bench sizes.
Usage (GPU box): python tools/time_resident.py [N,M,B[,K] ...]"""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "admm-deconv_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import admm_deconv  # noqa: E402
from admm_deconv import _lib, synth  # noqa: E402

# NAME=VALUE arguments are library options (admm_set_option), e.g. RESIDENT=2
for _a in [a for a in sys.argv[1:] if "=" in a]:
    _lib.set_option(_a.split("=")[0].upper(), int(_a.split("=")[1]))
    sys.argv.remove(_a)
TIME_ONLY = "--time-only" in sys.argv
if TIME_ONLY:
    sys.argv.remove("--time-only")
ISO = "--iso" in sys.argv          # the isotropic solve (resident_iso_kernel vs the 2-pass isotropic kernels)
if ISO:
    sys.argv.remove("--iso")
SHAPES = [(250, 250, 256, 25)]
if len(sys.argv) > 1:
    SHAPES = [tuple(int(v) for v in (a.split(",") + ["25"])[:4]) for a in sys.argv[1:]]


def solve(y, h, K, resident):
    with _lib.option("RESIDENT", 2 * int(resident)), _lib.option("MIN_PLANES", 0):   # 2: every compiled shape, any batch
        x = admm_deconv.tvd_fft(y, synth.LAMBDA, synth.RHO, h, ISO, K)
    torch.cuda.synchronize()
    return x


def rel(a, b):
    a = a.double().cpu().numpy()
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm((a - b).ravel()) / np.linalg.norm(b.ravel()))


def main():
    import oracle_np
    dev = torch.device("cuda", 0)
    out = []
    for N, M, B, K in SHAPES:
        hp = synth.gaussian_psf(15, 2.5)
        h = torch.from_numpy(hp).to(dev)
        # parity on 2 planes at a short K and the full K
        for k_chk, with_h in (() if TIME_ONLY else ((3, True), (K, True), (4, False))):
            yb = synth.make_batch(2, M, N, hp if with_h else None)
            y = torch.from_numpy(yb).to(dev)
            hh = h if with_h else None
            a = solve(y, hh, k_chk, True)
            b = solve(y, hh, k_chk, False)
            ref = oracle_np.to_c(oracle_np.tvd_fft_spectral(oracle_np.from_c(yb.astype(np.float64)),
                                                            np.float32(synth.LAMBDA), np.float32(synth.RHO),
                                                            oracle_np.psf_from_c(hp if with_h else None), ISO, k_chk))
            r = {"shape": [N, M], "K": k_chk, "psf": with_h, "resident_vs_2pass": rel(a, b.cpu().numpy()),
                 "resident_vs_oracle": rel(a, ref), "2pass_vs_oracle": rel(b, ref),
                 "finite": bool(torch.isfinite(a).all())}
            print(json.dumps(r), flush=True)
            out.append(r)
        y = torch.from_numpy(synth.make_batch(min(B, 8), M, N, hp)).to(dev)
        y = y.repeat((B + 7) // 8, 1, 1, 1)[:B].contiguous()
        for res in ((True,) if TIME_ONLY else (True, False)):
            for _ in range(2):
                solve(y, h, K, res)
            reps = 5
            t0 = time.perf_counter()
            with _lib.option("RESIDENT", 2 * int(res)), _lib.option("MIN_PLANES", 0):
                for _ in range(reps):
                    admm_deconv.tvd_fft(y, synth.LAMBDA, synth.RHO, h, ISO, K)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / reps
            _lib.profile_reset()
            _lib.profile_enable(True)
            solve(y, h, K, res)
            _lib.profile_enable(False)
            ks = {}
            for cls, name in _lib.KERNEL_CLASSES.items():
                ms, n = _lib.profile_get(cls)
                if n:
                    ks[name] = [round(ms, 4), n]
            r = {"shape": [N, M], "batch": B, "K": K, "iso": ISO, "resident": res, "ms": round(1000 * dt, 3),
                 "img_s": round(B / dt, 1), "kernel_ms_launches": ks}
            print(json.dumps(r), flush=True)
            out.append(r)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(REPO, "gpurun_out", "time_resident.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
