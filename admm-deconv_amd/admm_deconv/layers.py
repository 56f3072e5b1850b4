"""ADMM deconvolution layers -- host-side mirror of /root/reference/src/layers/deconv_admm.jl.

The reference defines four Flux layer types that differ only in which of (PSF weight, bias, λ, ρ)
are trainable (`Flux.@layer ... trainable=`, deconv_admm.jl:55,107,161,209) and share one forward
(deconv_admm.jl:215-225):

    d.λ = clamp.(d.λ, d.creg, Inf32);  d.ρ = clamp.(d.ρ, d.creg, Inf32)   # written back
    d.weight = clamp.(d.weight, 0f0, 1f0)                                   # written back
    res = tvd_fft(x, d.λ, d.ρ, d.weight, d.iso, d.iters) .+ d.bias
    return d.σ.(res)

Here the parameters are torch tensors on a ROCm device and `tvd_fft` is the HIP solve behind the
C ABI.  Shapes follow the rule "torch shape = reversed Julia shape": Julia weight (kh,kw,1,1) is
torch (1,1,kw,kh); Julia input (M,N,P,B) is torch (B,P,N,M).  λ and ρ stay on the device: the
projection clamps them in place there and the solve reads them in-kernel (admm_tvd_forward_dev_f32),
so neither the forward nor the backward reads them back to the host.  Under autograd the layer is
differentiable in (x, weight, λ, ρ) through the HIP adjoint of the K unrolled iterations (what Zygote
computes for the reference's training step, src/train.jl:51; BASELINE config c5).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .ops import multi_supported, tvd_fft, tvd_fft_multi_grad

__all__ = ["ADMMDeconv", "ADMMDeconvF1", "ADMMDeconvF2", "ADMMDeconvF3", "Admm", "Parallel", "chcat",
           "glorot_uniform", "identity", "relu", "relu6", "relu1"]


def identity(x):
    return x


def relu(x):
    return torch.relu(x)


class _ClampFn(torch.autograd.Function):
    """clamp(x, lo, hi) whose gradient is one HIP pass (admm_clamp_backward_f32: dy where lo <= x <= hi, as torch's
    clamp) instead of autograd's compare / compare / and / where kernels."""

    @staticmethod
    def forward(ctx, x, lo, hi):
        ctx.save_for_backward(x)
        ctx.lo, ctx.hi = lo, hi
        return torch.clamp(x, lo, hi)

    @staticmethod
    def backward(ctx, dy):
        from . import _lib
        (x,) = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        _lib.check(_lib.load().admm_clamp_backward_f32(x.data_ptr(), dy.data_ptr(), dx.data_ptr(), x.numel(),
                                                       float(ctx.lo), float(ctx.hi),
                                                       torch.cuda.current_stream(x.device).cuda_stream))
        return dx, None, None


def _clamp(x, lo, hi):
    if isinstance(x, torch.Tensor) and x.is_cuda and x.dtype == torch.float32 and x.is_contiguous() and x.requires_grad:
        return _ClampFn.apply(x, lo, hi)
    return torch.clamp(x, lo, hi)


def relu6(x):
    return _clamp(x, 0.0, 6.0)


def relu1(x):
    """relu1(x) = min.(relu.(x), 1) (src/nets/net_build.jl:8)."""
    return _clamp(x, 0.0, 1.0)


def _nfan(dims):
    """Flux.nfan: (fan_in, fan_out) for vector / matrix / conv-filter shapes (Julia order)."""
    if len(dims) == 1:
        return 1, dims[0]
    if len(dims) == 2:
        return dims[1], dims[0]
    k = math.prod(dims[:-2])
    return k * dims[-2], k * dims[-1]


def glorot_uniform(*dims_julia, rng=None):
    """Flux.glorot_uniform: (rand - 0.5) * sqrt(24 / (fan_in + fan_out)), float32, Julia dims.
    Returns a numpy array in torch/C order (reversed dims)."""
    rng = rng if rng is not None else np.random.default_rng()
    fi, fo = _nfan(dims_julia)
    a = (rng.random(tuple(reversed(dims_julia)), dtype=np.float64).astype(np.float32) - np.float32(0.5))
    return (a * np.float32(math.sqrt(24.0 / (fi + fo)))).astype(np.float32)


class Admm:
    """Shared state and forward of the four ADMM layer types (`Admm` union, deconv_admm.jl:212)."""
    TRAINABLE: tuple = ()

    def __init__(self, sigma, weight, bias, lam, rho, iters, iso, creg, device=None):
        dev = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        as_t = lambda v: torch.as_tensor(np.asarray(v, dtype=np.float32).reshape(-1), device=dev)  # noqa: E731
        self.sigma = sigma if sigma is not None else identity
        self.weight = torch.as_tensor(np.asarray(weight, dtype=np.float32), device=dev)
        self.bias = False if bias is False or bias is None else as_t(bias)
        self.lam = as_t(lam)
        self.rho = as_t(rho)
        self.iters = int(iters)
        self.iso = bool(iso)
        self.creg = float(creg)
        # torch.distributed group the batch is sharded over (isotropic prox: the pixelnorm spans the
        # whole sharded batch, see ops.tvd_fft); None = this process holds the whole batch
        self.group = None

    # Flux.@layer ... trainable=(...)
    def trainable(self):
        return {name: getattr(self, name) for name in self.TRAINABLE}

    @classmethod
    def from_params(cls, w, sigma, b, lam, rho, iters, iso, creg, device=None):
        """Positional constructor (deconv_admm.jl:18-28, :70-80, :122-132, :176-186)."""
        return cls.__new__(cls)._init_raw(sigma, w, b, lam, rho, iters, iso, creg, device)

    def _init_raw(self, *a, **k):
        Admm.__init__(self, *a, **k)
        return self

    def to(self, device):
        dev = torch.device(device)
        self.weight = self.weight.to(dev)
        self.lam = self.lam.to(dev)
        self.rho = self.rho.to(dev)
        if self.bias is not False:
            self.bias = self.bias.to(dev)
        return self

    def project(self):
        """The projection the forward writes back into the layer (deconv_admm.jl:216-219); in place on
        the leaf parameters so that, like Zygote on the reference, gradients reach the stored tensors."""
        with torch.no_grad():
            self.lam.clamp_(min=self.creg)                       # :216
            self.rho.clamp_(min=self.creg)                       # :217
            self.weight.clamp_(0.0, 1.0)                         # :219

    def __call__(self, x, scalars=None):
        """(d::Admm)(x) -- deconv_admm.jl:215-225.  λ and ρ are passed to the solve as device tensors
        (read in-kernel, no host sync).  scalars: optional host (lambda, rho) of the already projected
        layer, used instead of the device values."""
        if scalars is None:
            self.project()
        h = self.weight if self.weight.numel() > 0 else None
        res = tvd_fft(x, self.lam, self.rho, h, self.iso, self.iters, group=self.group, scalars=scalars)   # :221
        if self.bias is not False:
            res = res + self.bias                                 # :222
        return self.sigma(res)                                    # :224

    def __repr__(self):
        k = tuple(reversed(self.weight.shape[-2:])) if self.weight.numel() else ()
        return f"{type(self).__name__}({k}, {self.iters}, iso={self.iso})"


def _psf(k, init, groups, rng):
    if len(k) == 0:
        return np.zeros((0,), np.float32)                          # empty(ones(1))
    kh, kw = k
    w = init(kh, kw, 1, 1, rng=rng) if init is glorot_uniform else np.asarray(init(kh, kw, 1, 1), np.float32)
    return np.asarray(w, np.float32).reshape(1, 1, kw, kh)


def _bias(bias):
    if bias is False or bias is None:
        return False                                               # Flux.create_bias(w, false, 1)
    if bias is True:
        return np.zeros(1, np.float32)
    return np.asarray(bias, np.float32).reshape(-1)


class ADMMDeconv(Admm):
    """ADMMDeconv(k, num_it, σ=identity; iso, init, groups, bias, creg) -- deconv_admm.jl:189-209.
    Trainable: weight, bias, λ, ρ; λ, ρ initialised abs.(glorot_uniform(1))."""
    TRAINABLE = ("weight", "bias", "lam", "rho")

    def __init__(self, k, num_it, sigma=identity, *, iso=False, init=glorot_uniform, groups=1, bias=False,
                 creg=0.0, rng=None, device=None):
        rng = rng if rng is not None else np.random.default_rng()
        w = _psf(tuple(k), init, groups, rng)
        lam = np.abs(glorot_uniform(1, rng=rng))
        rho = np.abs(glorot_uniform(1, rng=rng))
        super().__init__(sigma, w, _bias(bias), lam, rho, num_it, iso, creg, device)


class ADMMDeconvF1(Admm):
    """ADMMDeconvF1(k, num_it, λ, σ; ...) -- fixed λ (deconv_admm.jl:31-55). Trainable: weight, bias, ρ."""
    TRAINABLE = ("weight", "bias", "rho")

    def __init__(self, k, num_it, lam, sigma=identity, *, iso=False, init=glorot_uniform, groups=1, bias=False,
                 creg=0.0, rng=None, device=None):
        assert lam > 0.0, "Parameter λ must be greater than 0"       # :42
        rng = rng if rng is not None else np.random.default_rng()
        w = _psf(tuple(k), init, groups, rng)
        rho = np.abs(glorot_uniform(1, rng=rng))
        super().__init__(sigma, w, _bias(bias), [lam], rho, num_it, iso, creg, device)


class ADMMDeconvF2(Admm):
    """ADMMDeconvF2(k, num_it, ρ, σ; ...) -- fixed ρ (deconv_admm.jl:83-107). Trainable: weight, bias, λ."""
    TRAINABLE = ("weight", "bias", "lam")

    def __init__(self, k, num_it, rho, sigma=identity, *, iso=False, init=glorot_uniform, groups=1, bias=False,
                 creg=0.0, rng=None, device=None):
        assert rho > 0, "Parameter ρ must be greater than 0"          # :94
        rng = rng if rng is not None else np.random.default_rng()
        w = _psf(tuple(k), init, groups, rng)
        lam = np.abs(glorot_uniform(1, rng=rng))
        super().__init__(sigma, w, _bias(bias), lam, [rho], num_it, iso, creg, device)


class ADMMDeconvF3(Admm):
    """ADMMDeconvF3(k, num_it, λ, ρ, σ; ...) -- fixed λ and ρ (deconv_admm.jl:135-161). Trainable: weight, bias."""
    TRAINABLE = ("weight", "bias")

    def __init__(self, k, num_it, lam, rho, sigma=identity, *, iso=False, init=glorot_uniform, groups=1,
                 bias=False, creg=0.0, rng=None, device=None):
        assert lam > 0, "Parameter λ must be greater than 0"          # :147
        assert rho > 0, "Parameter ρ must be greater than 0"          # :148
        rng = rng if rng is not None else np.random.default_rng()
        w = _psf(tuple(k), init, groups, rng)
        super().__init__(sigma, w, _bias(bias), [lam], [rho], num_it, iso, creg, device)


def chcat(*xs):
    """chcat(x...) = cat(x..., dims=3) (src/nets/net_build.jl:6): the channel axis, torch dim 1."""
    return torch.cat(xs, dim=1)


# isotropic branches are merged into one grid by default up to this many planes in all (c5 iso, 5 branches of
# 3-channel images: 30 planes 229 vs 119 img/s, 120: 730 vs 431, 240: 954 vs 740, 480: 984 vs 980, 960: 1027
# vs 1111 merged vs per-branch streams; profiles/r04_c5_configs.jsonl, profiles/r04_c5iso_merge.jsonl)
ISO_MERGE_MAX_PLANES = 512


class Parallel:
    """Flux `Parallel(connection, layers...)` as the nets build it (net_build.jl:121-125, :175): every
    branch sees the same input and `connection` combines the branch outputs.

    When every branch is an ADMM layer the one-grid solve covers (the denoiser: ADMMDeconvF2((), K, ρ_i, σ),
    256 x 256, same K and prox; isotropic when no ρ needs a gradient and the branches' planes fit one wave of
    workgroups, ISO_MERGE_MAX_PLANES, or with merge="always"), all branches run as ONE solve (ops.tvd_fft_multi: every branch's
    planes in one grid -- of the fused kernels, or below the library's plane-count rule (96 / 112 planes in all) of
    the 2-pass kernels -- the output already in the chcat layout) and one reverse sweep; each branch's bias and σ
    then apply to its slice.  The forward output, λ̄ and ρ̄ are bitwise those of the branches run one by one
    through the same kernels (tests/test_gpu_multi.py); when the merged grid is at or above the rule and a branch
    alone below it (e.g. 5 branches x 24 planes), the two run different kernels and agree to fp32 rounding, not
    bitwise (tests/test_gpu_default_rule.py).
    The input gradient matches to fp32 rounding in either case (branch_sum_kernel adds the branches' ȳ in a
    fixed order, not in autograd's per-branch accumulation order).  Otherwise the branches are independent, so on a ROCm device each runs on its own HIP stream
    (forward, and -- autograd replays a backward op on its forward's stream -- the adjoint too), then the
    caller's stream waits for all of them.  merge=False keeps the per-branch path; streams=False runs the
    branches one after the other on the caller's stream (the reference's single task-local stream)."""

    def __init__(self, connection, *layers, streams=True, merge=True):
        self.connection = connection
        self.layers = list(layers)
        self.use_streams = bool(streams)
        self.merge = merge if merge == "always" else bool(merge)
        self._streams = {}

    def _mergeable(self, x):
        if not self.merge or len(self.layers) < 2:
            return False
        Ls = self.layers
        if not all(isinstance(L, Admm) for L in Ls):
            return False
        K, iso = Ls[0].iters, Ls[0].iso
        # isotropic: its one-grid solve is a launch per iteration either way.  Up to ISO_MERGE_MAX_PLANES planes in
        # all (about two waves of workgroups, one plane per CU), one grid per iteration halves the launches and
        # fills the chip better: the reference's training batch (train_cfg.json batch_size 2, 5 branches x 6
        # planes) runs 229 img/s merged against 119 per-branch (417 since round 5: below the plane-count rule the
        # merged grid runs the 2-pass kernels).  Above that, the branches on their own streams
        # overlap one branch's batch-norm launches with the others' plane launches: batch 64 (960 planes) 1.11k
        # img/s per-branch against 1.03k merged.  merge="always" merges at any size.  The merged grid forms no
        # rho_bar.
        if iso:
            if any(self._needs_rho(L) for L in Ls):
                return False
            if self.merge != "always" and len(Ls) * x.shape[0] * x.shape[1] > ISO_MERGE_MAX_PLANES:
                return False
        return all(L.iters == K and L.iso == iso and L.weight.numel() == 0 and L.group is None for L in Ls) and \
            multi_supported(x, iso)

    @staticmethod
    def _needs_rho(L):
        return torch.is_grad_enabled() and isinstance(L.rho, torch.Tensor) and L.rho.requires_grad

    def _merged(self, x):
        """All branches in one solve (ops.tvd_fft_multi); bias and σ per branch, then the connection."""
        Ls = self.layers
        for L in Ls:
            L.project()          # deconv_admm.jl:216-219, in place on the device
        xa = tvd_fft_multi_grad(x, [L.lam for L in Ls], [L.rho for L in Ls], Ls[0].iters, Ls[0].iso)
        P = x.shape[1]
        if self.connection is chcat and all(L.bias is False and L.sigma is Ls[0].sigma for L in Ls):
            return Ls[0].sigma(xa)   # σ elementwise over the whole chcat tensor: the same values, no copies
        outs = []
        for i, L in enumerate(Ls):
            o = xa[:, i * P:(i + 1) * P]
            if L.bias is not False:
                o = o + L.bias
            outs.append(L.sigma(o))
        return self.connection(*outs)

    def _side_streams(self, dev):
        if dev not in self._streams:
            self._streams[dev] = [torch.cuda.Stream(device=dev) for _ in self.layers]
        return self._streams[dev]

    def __call__(self, x):
        if self._mergeable(x):
            return self._merged(x)
        if not (self.use_streams and isinstance(x, torch.Tensor) and x.is_cuda and len(self.layers) > 1):
            return self.connection(*[L(x) for L in self.layers])
        cur = torch.cuda.current_stream(x.device)
        side = self._side_streams(x.device)
        # each ADMM branch projects its λ / ρ / PSF in place on its own stream and the solve reads them
        # in-kernel: nothing here waits for the device
        outs = []
        for L, st in zip(self.layers, side):
            x.record_stream(st)     # read on st (forward, and by the adjoint on st after the join)
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                outs.append(L(x))
        for o, st in zip(outs, side):
            cur.wait_stream(st)
            o.record_stream(cur)    # allocated on st, consumed on the caller's stream
        return self.connection(*outs)

    def __getitem__(self, i):
        return self.layers[i]

    def __len__(self):
        return len(self.layers)

    def __repr__(self):
        return f"Parallel({getattr(self.connection, '__name__', self.connection)}, {', '.join(map(repr, self.layers))})"
