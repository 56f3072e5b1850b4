// Microbenchmark helper: a kernel that occupies `nblk` workgroups for `ticks` of the 100 MHz realtime
// clock, standing in for the few resident blocks an RCCL p2p kernel keeps on a rank while a gather is in
// flight.  tools/contend.py launches it beside the fused plane solve to see what a foreign resident
// workgroup costs a kernel that needs a whole CU per workgroup.
#include <hip/hip_runtime.h>

__global__ void hog_kernel(unsigned long long ticks, float* sink) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    float acc = (float)threadIdx.x;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
        acc = acc * 1.0001f + 1.0f;
        __builtin_amdgcn_s_sleep(2);
    }
    if (acc == -1.0f) sink[threadIdx.x] = acc;   // never taken; keeps the loop's VALU work live
}

extern "C" int launch_hog(int nblk, int nthreads, unsigned long long ticks, float* sink, void* stream) {
    if (nblk < 1 || nthreads < 64 || nthreads > 1024) return -1;
    hipLaunchKernelGGL(hog_kernel, dim3(nblk), dim3(nthreads), 0, (hipStream_t)stream, ticks, sink);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
