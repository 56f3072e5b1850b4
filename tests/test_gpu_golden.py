"""GPU vs the committed golden fixtures (fp64 oracle outputs) through the C ABI."""
import glob
import json
import os

import numpy as np
import pytest
import torch

import admm_deconv
from parity import assert_parity

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "*.npz"))), ids=os.path.basename)
def test_gpu_matches_fixture(dev, path):
    d = np.load(path)
    p = json.loads(str(d["params"]))
    y = torch.from_numpy(d["y"]).to(dev)
    h = torch.from_numpy(d["h"]).to(dev) if d["h"].size else None
    pow2 = lambda n: n & (n - 1) == 0  # noqa: E731
    if not (pow2(p["M"]) and pow2(p["N"])):
        with pytest.raises(admm_deconv.AdmmError) as e:
            admm_deconv.tvd_fft(y, p["lam"], p["rho"], h, p["iso"], p["K"])
        assert e.value.code == -2   # ADMM_E_UNSUPPORTED (non-power-of-two: SURVEY.md s8f next step)
        return
    x = admm_deconv.tvd_fft(y, p["lam"], p["rho"], h, p["iso"], p["K"])
    torch.cuda.synchronize()
    assert_parity(x.cpu().numpy(), d["x"], what=os.path.basename(path))
