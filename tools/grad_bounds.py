"""Measure the adjoint's gradient error against the fp64 autograd oracle next to the error of an fp32
autograd of the same oracle (what an fp32 implementation of the reference's Zygote pass gets), for
the backward test cases.  The GPU tolerances in tests/test_gpu_backward.py are set from this:
scalar gradients (lambda_bar, rho_bar, h_bar) must stay within SCALE x the fp32-autograd error plus a
floor.  Usage (GPU box): python tools/grad_bounds.py > gpurun_out/grad_bounds.txt"""
import os
import sys

import numpy as np
import torch

R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(R, "admm-deconv_amd"), os.path.join(R, "oracle"), os.path.join(R, "tests")]
import admm_deconv  # noqa: E402
import oracle_torch  # noqa: E402
from admm_deconv import synth  # noqa: E402
from test_gpu_backward import CASES, FUSED_ADJ_CASES, psf  # noqa: E402


def rel(a, b):
    return abs(a - b) / max(abs(b), 1e-12)


def main():
    dev = torch.device("cuda", 0)
    rows = []
    for B, P, N, M, spec, lam, rho, K, _ in CASES:
        rows.append(("2pass/bwd", B, P, N, M, spec, lam, rho, K, 11, N + M + K))
    for B, P, spec, lam, rho, K in FUSED_ADJ_CASES:
        rows.append(("fused-adj", B, P, 256, 256, spec, lam, rho, K, 21, K + 17 * B))
    for kind, B, P, N, M, spec, lam, rho, K, g0, seed in rows:
        rng = np.random.default_rng(seed)
        h = psf(spec, rng)
        y = synth.make_batch(B, M, N, h, P=P, g0=g0)
        xbar = rng.standard_normal(y.shape).astype(np.float32)
        ht = None if h is None else torch.from_numpy(h).to(dev)
        need_h = h is not None and kind != "fused-adj"
        _, yb, hb, lb, rb = admm_deconv.tvd_fft_backward(torch.from_numpy(y).to(dev), torch.from_numpy(xbar).to(dev),
                                                         lam, rho, ht, False, K, need_h=need_h)
        torch.cuda.synchronize()
        h64 = None if h is None else h.astype(np.float64)
        r64 = oracle_torch.tvd_fft_grads(y.astype(np.float64), np.float32(lam), np.float32(rho), h64, False, K, xbar)
        r32 = oracle_torch.tvd_fft_grads(y, np.float32(lam), np.float32(rho), h, False, K, xbar, dtype=torch.float32)
        line = (f"{kind} {B}x{P}x{N}x{M} {spec} K={K}: lam gpu {rel(float(lb), r64[3]):.2e} fp32 {rel(r32[3], r64[3]):.2e}"
                f" | rho gpu {rel(float(rb), r64[4]):.2e} fp32 {rel(r32[4], r64[4]):.2e}")
        if need_h:
            e = np.linalg.norm(hb.cpu().numpy() - r64[2]) / np.linalg.norm(r64[2])
            e32 = np.linalg.norm(r32[2] - r64[2]) / np.linalg.norm(r64[2])
            line += f" | hbar gpu {e:.2e} fp32 {e32:.2e}"
        ey = np.linalg.norm(yb.cpu().numpy().astype(np.float64) - r64[1]) / np.linalg.norm(r64[1])
        ey32 = np.linalg.norm(r32[1].astype(np.float64) - r64[1]) / np.linalg.norm(r64[1])
        line += f" | ybar gpu {ey:.2e} fp32 {ey32:.2e}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
