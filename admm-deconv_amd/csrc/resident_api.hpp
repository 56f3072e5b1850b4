// resident_api.hpp -- host entry points of admm_resident.hip: the whole K-iteration anisotropic solve of
// one plane per workgroup for the smooth non-power-of-two shapes this build compiled (sides <= 256).
// Same buffers and results as the smooth 2-pass path (admm_smooth.hip) it replaces.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

namespace admm {
namespace rs {

// M = line length (contiguous), N = lines; true if this build has a resident kernel for M x N (all = false:
// only where it measured faster than the 2-pass kernels)
bool has_shape(int M, int N, bool all = false);
// hty: H^T y per plane (or y itself without a PSF); s ping-pong buffers sA / sB ([plane][2][N][M]) unless
// traj != nullptr (then s_k goes to traj + (k - 1) * traj_stride, read back from the previous slot);
// Ct / twM / twN / prm: the setup kernel's tables; stagger: start delay per workgroup group (realtime ticks,
// ADMM_OPT_PLANE_STAGGER).  Returns -1 when the shape is not compiled.
int launch(int M, int N, size_t planes, hipStream_t s, const float* hty, float* sA, float* sB, float* traj,
           size_t traj_stride, float* x_out, const float* Ct, const float2* twM, const float2* twN, const float* prm,
           int maxit, int stagger = 0);

}  // namespace rs
}  // namespace admm
