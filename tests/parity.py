"""Parity criterion (SURVEY.md s7 'Hard parts', s8c): per-plane relative L2 <= 1e-5 against the fp64
oracle on identical fp32 inputs, plus a max-abs guard <= 2e-4 * max|ref|."""
import numpy as np

REL_L2_TOL = 1e-5
MAXABS_TOL = 2e-4


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
