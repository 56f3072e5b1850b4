import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "admm-deconv_amd")
for p in (os.path.join(REPO, "admm-deconv_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: longer CPU test")
    config.addinivalue_line("markers", "min_planes_rule: GPU test run with the library's plane-count path rule "
                            "(ADMM_OPT_MIN_PLANES at its default) instead of per-plane kernels at every batch")


@pytest.fixture(autouse=True)
def _per_plane_paths_at_every_batch(request):
    """GPU tests solve small batches but mean the per-plane kernels (fused / resident) wherever the path table
    names them, as tests/paths_table.py does: the plane-count rule (ADMM_OPT_MIN_PLANES, which leaves small
    batches to the 2-pass kernels) is off for them, unless a test is marked min_planes_rule.  Multi-process GPU
    tests set the same option in their workers."""
    if request.node.get_closest_marker("gpu") is None or request.node.get_closest_marker("min_planes_rule"):
        yield
        return
    from admm_deconv import _lib
    with _lib.option("MIN_PLANES", 0):
        yield


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
