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
// the same for the isotropic solve (launch_iso)
bool has_iso_shape(int M, int N, bool all = false);
// hty: H^T y per plane (or y itself without a PSF); s ping-pong buffers sA / sB ([plane][2][N][M]) unless
// traj != nullptr (then s_k goes to traj + (k - 1) * traj_stride, read back from the previous slot);
// Ct / twM / twN / prm: the setup kernel's tables.  Returns -1 when the shape is not compiled.
int launch(int M, int N, size_t planes, hipStream_t s, const float* hty, float* sA, float* sB, float* traj,
           size_t traj_stride, float* x_out, const float* Ct, const float2* twM, const float2* twN, const float* prm,
           int maxit);

// The isotropic solve's iteration k (0 .. K-1) as one launch (admm_resident.hip resident_iso_kernel): reads s_k
// (s_in, k > 0) and f_k (fmap, M x N), writes s_{k+1} (s_out; may equal s_in) and q = s1^2 + s2^2 per plane
// (q: planes x M x N) for the caller's norm kernel, or x at k = K - 1.  Returns -1 when the shape is not
// compiled.
int launch_iso(int M, int N, size_t planes, hipStream_t s, const float* hty, const float* s_in, float* s_out,
               const float* fmap, float* q, float* x_out, const float* Ct, const float2* twM, const float2* twN,
               const float* prm, int k, int K);

}  // namespace rs
}  // namespace admm
