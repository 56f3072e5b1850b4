"""Seeded synthetic deconvolution inputs.

Per image with GLOBAL index g (so a batch sharded over ranks is bit-identical to the unsharded
batch): a counter-based splitmix64 stream seeded with 20241008 + g draws 20 axis-aligned
rectangles (side U{4..dim/3}, value U[0,1]) on a zero background; the image is blurred by the
centred circular convolution H of the reference (ops.jl:80) with a normalised Gaussian PSF, and
AWGN (sigma 0.01) is added.  Values are not clamped.  Planes of an RGB image use g*P + p.
Generation is host-side numpy and is never inside a timed region.
"""
from __future__ import annotations

import numpy as np

SEED0 = 20241008
_GOLD = np.uint64(0x9E3779B97F4A7C15)
_C1 = np.uint64(0xBF58476D1CE4E5B9)
_C2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed, counters):
    """Counter-based splitmix64: the n-th output of the stream seeded with `seed`."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (np.asarray(counters, dtype=np.uint64) + np.uint64(1)) * _GOLD
        z = (z ^ (z >> np.uint64(30))) * _C1
        z = (z ^ (z >> np.uint64(27))) * _C2
        return z ^ (z >> np.uint64(31))


def uniform(seed, counters):
    return (splitmix64(seed, counters) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def gaussian_psf(k, sigma):
    """Normalised k x k Gaussian PSF in C layout (kw, kh) (== Julia (kh, kw); symmetric)."""
    a = np.arange(k) - (k - 1) / 2.0
    g = np.exp(-(a * a) / (2.0 * sigma * sigma))
    p = np.outer(g, g)
    return (p / p.sum()).astype(np.float32)


def box_psf_row(k=7):
    """The reference test's PSF: 7x7 zeros with row 4 = 1/7 (src/tests/admm_deconv_test.jl:19-20).
    Julia blur_psf[4, :] is dim1 index 4 -> C layout (kw, kh) column a=3 over all b."""
    p = np.zeros((k, k), np.float32)
    p[:, k // 2] = 1.0 / k
    return p


def ground_truth(g, M, N, nrect=20):
    seed = SEED0 + int(g)
    u = uniform(seed, np.arange(5 * nrect)).reshape(nrect, 5)
    img = np.zeros((N, M), np.float64)
    for r in range(nrect):
        w = 4 + int(u[r, 0] * max(M // 3 - 3, 1))
        h = 4 + int(u[r, 1] * max(N // 3 - 3, 1))
        i0 = int(u[r, 2] * M)
        j0 = int(u[r, 3] * N)
        img[j0:j0 + h, i0:i0 + w] = u[r, 4]
    return img


def blur(img, psf_c):
    """Centred circular convolution H (ops.jl:80) of a (N, M) image with PSF (kw, kh), via FFT."""
    N, M = img.shape
    kw, kh = psf_c.shape
    padd, padr = (kh - 1) // 2, (kw - 1) // 2
    k = np.zeros((N, M))
    for b in range(kw):
        for a in range(kh):
            k[(b - padr) % N, (a - padd) % M] += psf_c[b, a]
    return np.real(np.fft.ifft2(np.fft.fft2(img) * np.fft.fft2(k)))


def noise(g, n, sigma=0.01):
    seed = SEED0 + int(g)
    c = 1000 + 2 * np.arange(n, dtype=np.uint64)
    u1 = 1.0 - uniform(seed, c)
    u2 = uniform(seed, c + np.uint64(1))
    return sigma * np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)


def make_clean(B, M, N, P=1, g0=0):
    """The ground-truth images of make_batch (no blur, no noise), float32 (B,P,N,M)."""
    out = np.empty((B, P, N, M), np.float32)
    for b in range(B):
        for p in range(P):
            out[b, p] = ground_truth((g0 + b) * P + p, M, N).astype(np.float32)
    return out


def make_batch(B, M, N, psf_c, P=1, g0=0, sigma=0.01):
    """float32 array (B, P, N, M) of blurred noisy images with global indices g0..g0+B-1."""
    out = np.empty((B, P, N, M), np.float32)
    for b in range(B):
        for p in range(P):
            g = (g0 + b) * P + p
            img = ground_truth(g, M, N)
            if psf_c is not None and np.size(psf_c):
                img = blur(img, psf_c)
            out[b, p] = (img + noise(g, M * N, sigma).reshape(N, M)).astype(np.float32)
    return out


# BASELINE.json configs
CONFIGS = {
    "c1": dict(M=64, N=64, P=1, B=1, psf=(9, 1.2), K=10),
    "c2": dict(M=256, N=256, P=1, B=512, psf=(15, 2.5), K=25),
    "c3": dict(M=256, N=256, P=1, B=2048, psf=(15, 2.5), K=25),
    "c4": dict(M=512, N=512, P=3, B=256, psf=(15, 2.5), K=50),
    # c5: the get_denoiser branch (src/nets/net_build.jl:113-128): 5 x ADMMDeconvF2((), 50, rho, relu1),
    # batch 64 of 256x256 RGB (train_cfg.json im_shape), forward + adjoint
    "c5": dict(M=256, N=256, P=3, B=64, psf=None, K=50),
}
LAMBDA, RHO = 0.0041, 0.021   # src/tests/admm_deconv_test.jl:76
