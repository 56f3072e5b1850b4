// scalar_src.hpp -- where a solve's lambda and rho come from (shared by the kernels and the host ABI).
#pragma once

namespace admm {

// device pointers (the reference's 1-element CuArrays, `tvd_fft(y, λ::CGPUArray, ρ::CGPUArray, ...)`,
// /root/reference/src/ops/ops.jl:99,181 -- read on the device, no host sync) or, when a pointer is NULL,
// the host value (admm_kernels.hip setup_kernel resolves them into the workspace's scalar block)
struct ScalarSrc {
    const float* lam;
    const float* rho;
    float lam_v;
    float rho_v;
};

}  // namespace admm
