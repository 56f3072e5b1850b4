"""admm_deconv -- MI355X-native ADMM TV deconvolution (drop-in for georgegrosu1/admm-deconv's
`tvd_fft` hot path and its Flux ADMM layers).

Package layout (the directory admm-deconv_amd/ is the product):
  csrc/            HIP kernels for gfx950 + the extern "C" boundary (include/admm_deconv.h)
  libadmm_deconv.so  built in-tree by __graft_entry__.build()
  admm_deconv/     host-side mirror of the reference interface:
     ops.py        tvd_fft            (src/ops/ops.jl:181); tvd_fft_multi (the branches of a
                   Parallel(chcat, ...) of ADMM layers in one grid, src/nets/net_build.jl:113-125)
     layers.py     ADMMDeconv, ADMMDeconvF1/F2/F3 (src/layers/deconv_admm.jl)
     synth.py      seeded synthetic blurred batches
     parallel.py   batch sharding over ranks + RCCL gather
"""
from ._lib import AdmmError, load, workspace_bytes  # noqa: F401
from .ops import (tvd_fft, tvd_fft_backward, tvd_fft_record, tvd_fft_backward_recorded, Recording,  # noqa: F401
                  Workspace, tvd_fft_multi, tvd_fft_multi_backward_recorded, MultiRecording)

__version__ = "0.1.0"
