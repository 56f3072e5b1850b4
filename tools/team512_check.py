"""Experiment check (round 5): the persistent team512 launch (ADMM_EXP_TEAM512=1, admm_kernels.hip team512_kernel)
against the 2-pass launches on the same inputs -- the same kernel bodies, so the outputs must be bitwise equal.
Runs the 2-pass solve in a child process without the switch (the switch is read once per process)."""
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "admm-deconv_amd"))


def solve(out, B, K):
    import torch
    import admm_deconv
    from admm_deconv import synth
    h = synth.gaussian_psf(15, 2.5)
    y = synth.make_batch(B, 512, 512, h, P=3, g0=5)
    dev = torch.device("cuda", 0)
    x = admm_deconv.tvd_fft(torch.from_numpy(y).to(dev), 0.0041, 0.021, torch.from_numpy(h).to(dev), False, K)
    torch.cuda.synchronize()
    np.save(out, x.cpu().numpy())


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        solve(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
        sys.exit(0)
    B, K = 96, 6   # 288 planes: more than one plane per team
    outs = {}
    for mode in ("2pass", "team"):
        env = dict(os.environ)
        env.pop("ADMM_EXP_TEAM512", None)
        if mode == "team":
            env["ADMM_EXP_TEAM512"] = "1"
        path = f"/tmp/team512_{mode}.npy"
        subprocess.run([sys.executable, __file__, "child", path, str(B), str(K)], env=env, check=True, timeout=300)
        outs[mode] = np.load(path)
    a, b = outs["2pass"], outs["team"]
    print("bitwise equal:", bool(np.array_equal(a, b)), "max abs diff:", float(np.abs(a - b).max()))
    sys.exit(0 if np.array_equal(a, b) else 1)
