"""Generate the golden fixtures in tests/golden/ from the fp64 oracle (oracle/oracle_np.py).

The reference ships no golden vectors; these fixtures pin the oracle's output on
fp32 inputs produced by admm_deconv.synth (seeded, counter-based), so the GPU tests can compare
against committed data as well as against a live oracle run.  Each fixture stores the float32 input
y (C layout (B,P,N,M)), the PSF h (C layout (kw,kh), possibly empty), the solver parameters and the
fp64 oracle output rounded to float32.

    python tests/golden/gen_golden.py          # rewrites tests/golden/*.npz and manifest.json
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "admm-deconv_amd"), os.path.join(REPO, "oracle")]

import oracle_np  # noqa: E402
from admm_deconv import synth  # noqa: E402

FIXTURES = [
    # name, B, P, N, M, psf, lam, rho, iso, K
    ("c1_64_k10", 1, 1, 64, 64, ("gauss", 9, 1.2), 0.0041, 0.021, False, 10),
    ("c2_256_k25_slices", 2, 1, 256, 256, ("gauss", 15, 2.5), 0.0041, 0.021, False, 25),
    ("iso_box7_64_k20", 4, 1, 64, 64, ("box",), 0.0041, 0.021, True, 20),
    ("even_psf10_64x128_k15", 2, 1, 128, 64, ("rand", 10, 10), 0.01, 0.05, False, 15),
    ("denoise_rgb_64_k30", 2, 3, 64, 64, None, 0.05, 0.02, False, 30),
    ("nonpow2_40x48_k5", 1, 1, 40, 48, ("gauss", 5, 1.0), 0.0041, 0.021, False, 5),
    # BASELINE c4 (512^2, 15x15 PSF, K = 50): one plane of the RGB batch (planes are independent)
    ("c4_512_k50_plane", 1, 1, 512, 512, ("gauss", 15, 2.5), 0.0041, 0.021, False, 50),
]


def psf_of(spec, seed):
    if spec is None:
        return np.zeros((0, 0), np.float32)
    if spec[0] == "gauss":
        return synth.gaussian_psf(spec[1], spec[2])
    if spec[0] == "box":
        return synth.box_psf_row(7)
    rng = np.random.default_rng(seed)
    h = rng.random((spec[2], spec[1])).astype(np.float32)
    return (h / h.sum()).astype(np.float32)


def main():
    manifest = {}
    for i, (name, B, P, N, M, psf, lam, rho, iso, K) in enumerate(FIXTURES):
        h = psf_of(psf, 100 + i)
        y = synth.make_batch(B, M, N, h if h.size else None, P=P, g0=1000 * i)
        x = oracle_np.to_c(oracle_np.tvd_fft_literal(oracle_np.from_c(y.astype(np.float64)), np.float32(lam),
                                                     np.float32(rho), oracle_np.psf_from_c(h) if h.size else None,
                                                     iso, K))
        params = dict(lam=lam, rho=rho, iso=iso, K=K, B=B, P=P, N=N, M=M, psf=list(psf) if psf else None)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), y=y, h=h, x=x.astype(np.float32),
                            params=np.array(json.dumps(params)))
        manifest[name] = params
        print(name, y.shape, h.shape, float(np.abs(x).max()))
    json.dump(manifest, open(os.path.join(HERE, "manifest.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
