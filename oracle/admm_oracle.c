/* CPU oracle / CPU baseline for the ADMM TV-deconvolution solve -- TEST INFRASTRUCTURE ONLY.
 *
 * A C restatement of /root/reference/src/ops/ops.jl:17-96 (`tvd_fft_cpu`), op for op (see
 * admm_oracle_impl.h).  Two precisions are exported:
 *   oracle_tvd_fft_f32  -- the reference's own arithmetic type (Float32); bench.py times this
 *                          on the GPU box's host cores as `cpu_baseline` (kind "port").
 *   oracle_tvd_fft_f64  -- cross-checks the numpy fp64 oracle (oracle_np.py).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product path (admm-deconv_amd/) never does.
 *
 * Parity status: parity unpinned (Julia reference absent; no reference golden vectors exist;
 * see oracle_np.py header and DESIGN.md).  FFTW (FFTW_jll 3.3.10, Manifest.toml:601-611) is
 * not installed, so this file carries its own radix-2 FFT (naive DFT for other lengths).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

#define R float
#define SFX f32
#include "admm_oracle_impl.h"
#undef R
#undef SFX

#define R double
#define SFX f64
#include "admm_oracle_impl.h"
#undef R
#undef SFX

int oracle_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
