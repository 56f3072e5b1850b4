"""Parity criterion (SURVEY.md s7 'Hard parts', s8c): per-plane relative L2 <= 1e-5 against the fp64
oracle on identical fp32 inputs, plus a max-abs guard <= 2e-4 * max|ref|.

Ill-conditioned inputs (a PSF spectrum with near-zeros, a prox live almost everywhere) put every fp32 solve
further than 1e-5 from the fp64 oracle.  For them the bound is the error of THE REFERENCE'S OWN ALGORITHM IN
FLOAT32 on the same inputs: oracle/admm_oracle.c is the op-for-op restatement of tvd_fft_cpu
(/root/reference/src/ops/ops.jl:17-96: per-iteration spatial H^T y, 2x2 stencils, FFT solve, ST / BT) in the
reference's Float32.  assert_parity_fp32ref: rel-L2 <= max(1e-5, that error), no other slack."""
import numpy as np

REL_L2_TOL = 1e-5
MAXABS_TOL = 2e-4
# a parity case pins the nonlinear part of the solve (ST/BT, /root/reference/src/ops/ops.jl:6-10, 89) only if
# the prox is live: at least this fraction of the oracle's prox outputs z_k (or, adjoint, of the recorded
# masks 1[|s_k| > tau]) must be non-zero, averaged over the iterations that reach the output
PROX_MIN_FRACTION = 0.01


def assert_prox_active(frac, what="", linear_only=False):
    """Every parity case either proves that its prox fired (frac >= PROX_MIN_FRACTION) or is declared a
    linear-only check (K = 1, tau above every |Dx|): then the prox must really be dead, so that the label
    cannot hide a case that was meant to be nonlinear."""
    if linear_only:
        assert frac == 0.0, f"{what}: declared linear-only but {frac:.3%} of prox outputs are live"
    else:
        assert frac >= PROX_MIN_FRACTION, (f"{what}: prox live in only {frac:.3%} of elements "
                                           f"(< {PROX_MIN_FRACTION:.0%}): the case checks only the linear solve")
    return frac


def oracle_solve(y, lam, rho, h, iso, K, form="literal", linear_only=False, what=""):
    """The fp64 oracle (oracle/oracle_np.py) on C-layout fp32 inputs y (B,P,N,M), h (kw,kh) or None, with lam and
    rho rounded to fp32 as the library takes them; asserts whether the prox fired (assert_prox_active)."""
    import oracle_np
    f = oracle_np.tvd_fft_literal if form == "literal" else oracle_np.tvd_fft_spectral
    st = {}
    x = oracle_np.to_c(f(oracle_np.from_c(np.asarray(y, np.float64)), np.float32(lam), np.float32(rho),
                         oracle_np.psf_from_c(h), iso, K, stats=st))
    if linear_only is not None:
        assert_prox_active(oracle_np.prox_active_fraction(st), what, linear_only)
    return x


def assert_parity(got, ref, rel_tol=REL_L2_TOL, maxabs_tol=MAXABS_TOL, what=""):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    assert np.all(np.isfinite(got)), f"{what}: non-finite output"
    planes_g = got.reshape(-1, got.shape[-2] * got.shape[-1])
    planes_r = ref.reshape(-1, ref.shape[-2] * ref.shape[-1])
    worst = 0.0
    for i in range(planes_g.shape[0]):
        nr = np.linalg.norm(planes_r[i])
        d = np.linalg.norm(planes_g[i] - planes_r[i])
        rel = d / nr if nr > 0 else d
        worst = max(worst, rel)
        assert rel <= rel_tol, f"{what}: plane {i} relative L2 {rel:.3e} > {rel_tol:.0e}"
    scale = max(np.abs(ref).max(), 1e-30)
    mx = np.abs(got - ref).max() / scale
    assert mx <= maxabs_tol, f"{what}: max-abs {mx:.3e} > {maxabs_tol:.0e} * max|ref|"
    return worst, mx


def assert_case_prox_active(y, lam, rho, h, iso, K, what="", linear_only=None):
    """assert_prox_active for a case checked against another oracle form (the autograd gradient oracle): the
    fraction comes from the fp64 spectral oracle's forward on the same inputs.  linear_only defaults to K == 1
    (the K-th prox output is dead, ops.jl:84-93)."""
    import oracle_np
    st = {}
    oracle_np.tvd_fft_spectral(oracle_np.from_c(np.asarray(y, np.float64)), np.float32(lam), np.float32(rho),
                               oracle_np.psf_from_c(h), iso, K, stats=st)
    return assert_prox_active(oracle_np.prox_active_fraction(st), what, K <= 1 if linear_only is None else linear_only)


def c_fp32_error(y, lam, rho, h, iso, K, ref):
    """(worst per-plane rel-L2, max-abs / max|ref|) of oracle/admm_oracle.c in float32 (the reference's CPU solve,
    ops.jl:17-96, in its own Float32) against the fp64 oracle's `ref` on the same fp32 inputs."""
    import oracle_c
    x32 = np.asarray(oracle_c.tvd_fft_c(np.asarray(y, np.float32), np.float32(lam), np.float32(rho), h, iso, K,
                                        np.float32), np.float64)
    ref = np.asarray(ref, np.float64)
    a = x32.reshape(-1, x32.shape[-2] * x32.shape[-1])
    b = ref.reshape(a.shape)
    rel = max(np.linalg.norm(a[i] - b[i]) / max(np.linalg.norm(b[i]), 1e-300) for i in range(a.shape[0]))
    return rel, float(np.abs(x32 - ref).max() / max(np.abs(ref).max(), 1e-30))


def assert_parity_fp32ref(got, ref, y, lam, rho, h, iso, K, what=""):
    """assert_parity at 1e-5; where that fails, the bound is the C fp32 reference solve's own error on the same
    inputs (module docstring) -- the GPU must be no further from the fp64 oracle than the reference's algorithm
    in float32 is.  Returns (worst rel-L2, max-abs, the fp32 reference's rel-L2 or None)."""
    try:
        w, m = assert_parity(got, ref, what=what)
        return w, m, None
    except AssertionError:
        e32, m32 = c_fp32_error(y, lam, rho, h, iso, K, ref)
        w, m = assert_parity(got, ref, rel_tol=max(REL_L2_TOL, e32), maxabs_tol=max(MAXABS_TOL, m32),
                             what=f"{what} (C fp32 reference solve: rel-L2 {e32:.2e}, max-abs {m32:.2e})")
        return w, m, e32
