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
    x = admm_deconv.tvd_fft(y, p["lam"], p["rho"], h, p["iso"], p["K"])
    torch.cuda.synchronize()
    assert_parity(x.cpu().numpy(), d["x"], what=os.path.basename(path))
