"""Time the runtime-length (generic-size) path on a few shapes: images/s and the canonical 2-pass
byte model of SURVEY.md s8d (32 (M/2+1) N + 20 M N bytes per plane-iteration) as GB/s.
Usage (GPU box): python tools/time_generic.py"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "admm-deconv_amd"))
import admm_deconv  # noqa: E402
from admm_deconv import _lib, synth  # noqa: E402

# NAME=VALUE arguments are library options (admm_set_option), e.g. FUSED=0 LINE_T=4 GEN_TM=4096
for _a in [a for a in sys.argv[1:] if "=" in a]:
    _lib.set_option(_a.split("=")[0].upper(), int(_a.split("=")[1]))
    sys.argv.remove(_a)

SHAPES = [(480, 640, 64, 25), (96, 96, 512, 25), (250, 250, 256, 25), (2048, 2048, 8, 25), (256, 256, 512, 25)]
# positional N,M,B[,K] arguments replace the default shape list (e.g. 250,250,256 for one rocprof run)
if len(sys.argv) > 1:
    SHAPES = [tuple(int(v) for v in (a.split(",") + ["25"])[:4]) for a in sys.argv[1:]]


def main():
    dev = torch.device("cuda", 0)
    h = torch.from_numpy(synth.gaussian_psf(15, 2.5)).to(dev)
    out = []
    for N, M, B, K in SHAPES:
        y = torch.from_numpy(synth.make_batch(min(B, 8), M, N, synth.gaussian_psf(15, 2.5))).to(dev)
        y = y.repeat((B + 7) // 8, 1, 1, 1)[:B].contiguous()
        for _ in range(2):
            admm_deconv.tvd_fft(y, synth.LAMBDA, synth.RHO, h, False, K)
        torch.cuda.synchronize()
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            admm_deconv.tvd_fft(y, synth.LAMBDA, synth.RHO, h, False, K)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        canon = B * (K * (32 * (M // 2 + 1) * N + 20 * M * N) + 12 * M * N)
        _lib.profile_reset()
        _lib.profile_enable(True)
        admm_deconv.tvd_fft(y, synth.LAMBDA, synth.RHO, h, False, K)
        _lib.profile_enable(False)
        ks = {}
        for cls, name in _lib.KERNEL_CLASSES.items():
            ms, n = _lib.profile_get(cls)
            if n:
                ks[name] = round(ms, 3)
        r = {"shape": [N, M], "batch": B, "K": K, "ms": round(1000 * dt, 3), "img_s": round(B / dt, 1),
             "canonical_GBps": round(canon / dt / 1e9, 1), "kernel_ms": ks,
             "path": _lib.query_paths(M, N, False, 15, planes=B)[0], "schedule": _lib.forward_schedule(M, N, False, 15, B)}
        print(json.dumps(r), flush=True)
        out.append(r)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open("gpurun_out/time_generic.json", "w"), indent=1)


if __name__ == "__main__":
    main()
