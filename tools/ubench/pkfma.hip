// Microbenchmark: issue rate of packed (v_pk_fma_f32 / v_pk_add_f32) vs scalar (v_fma_f32 / v_add_f32)
// FP32 VALU on gfx950.  Each thread runs 16 independent chains for `iters` iterations.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

__global__ void k_pk_fma(float* out, int iters, float a, float b) {
    f2 v[16];
    for (int i = 0; i < 16; ++i) v[i] = f2{(float)threadIdx.x + i, (float)i};
    const f2 A = {a, a}, B = {b, b};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = __builtin_elementwise_fma(v[i], A, B);
    }
    float s = 0;
    for (int i = 0; i < 16; ++i) s += v[i].x + v[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_fma(float* out, int iters, float a, float b) {
    float v[32];
    for (int i = 0; i < 32; ++i) v[i] = (float)threadIdx.x + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 32; ++i) v[i] = __builtin_fmaf(v[i], a, b);
    }
    float s = 0;
    for (int i = 0; i < 32; ++i) s += v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_pk_add(float* out, int iters, float a, float b) {
    f2 v[16];
    for (int i = 0; i < 16; ++i) v[i] = f2{(float)threadIdx.x + i, (float)i};
    const f2 A = {a, b};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = v[i] + A;
    }
    float s = 0;
    for (int i = 0; i < 16; ++i) s += v[i].x + v[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_add(float* out, int iters, float a, float b) {
    float v[32];
    for (int i = 0; i < 32; ++i) v[i] = (float)threadIdx.x + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 32; ++i) v[i] = v[i] + (i & 1 ? a : b);
    }
    float s = 0;
    for (int i = 0; i < 32; ++i) s += v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
void run(const char* name, K k, float* d, int blocks, int threads, int iters, double flops_per_iter_thread) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 10, 1.0001f, 0.5f);
    hipEventRecord(a);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, iters, 1.0001f, 0.5f);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    double fl = flops_per_iter_thread * iters * (double)blocks * threads;
    printf("%-8s blocks %5d x %4d: %.3f ms  %.1f TFLOP/s  (%.2f G wave-instr/s per CU)\n", name, blocks, threads, ms,
           fl / ms / 1e9, 0.0);
}

int main() {
    float* d;
    hipMalloc(&d, 1 << 26);
    for (int bl : {1024, 4096}) {
        run("pk_fma", k_pk_fma, d, bl, 256, 20000, 16 * 4);
        run("fma", k_fma, d, bl, 256, 20000, 32 * 2);
        run("pk_add", k_pk_add, d, bl, 256, 20000, 16 * 2);
        run("add", k_add, d, bl, 256, 20000, 32);
    }
    return 0;
}
