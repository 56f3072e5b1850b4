// smooth_api.hpp -- host entry points of admm_smooth.hip (the runtime-length path's per-iteration
// kernels with compile-time plans for the lengths listed there).  Same buffers and semantics as the
// admm_generic.hip kernels they replace; each launcher returns -1 when the length is not compiled.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

namespace admm {
namespace sm {

bool has_length(int n);   // a line length M or column length N this build compiled
int line_lines(int M);    // lines per line block (0 if not compiled)
int column_slots(int N);  // spectral columns per column block (0 if not compiled)
size_t line_lds(int M);
size_t column_lds(int N);

// spec (N x (M/2+1) per plane) -> dim-2 FFT, x multiplier, IFFT -> dst (gen::column_kernel modes 0 / 1):
// mul 0: cs * Ct, mul 1: Gt (H^T);  mode = ADMM_OPT_SMOOTH (1: measured plan order per length, 2 / 3:
// increasing / decreasing radices); yh (not NULL): + Y_h = F(H^T y) before the multiply (gen::column_kernel mode 16)
int launch_column(int M, int N, size_t planes, hipStream_t s, const float2* src, float2* dst, const float* Ct,
                  const float2* Gt, const float2* twN, float cs, int mul, int mode, const float2* yh = nullptr);
// (line_upd: hty NULL = H^T y enters spectrally, v = rho D^T w)
// real lines -> half spectra (gen::line_fwd_kernel)
int launch_line_fwd(int M, int N, size_t planes, hipStream_t s, const float* src, float2* spec, const float2* twM);
// half spectra -> real lines (gen::line_inv_kernel)
int launch_line_inv(int M, int N, size_t planes, hipStream_t s, const float2* spec, float* dst, const float2* twM);
// anisotropic line update + forward transform (gen::line_upd_kernel)
int launch_line_upd(int M, int N, size_t planes, hipStream_t s, const float* x, const float* s_old, float* s_new,
                    const float* hty, float2* spec, const float2* twM, const float* prm, int first);

}  // namespace sm
}  // namespace admm
