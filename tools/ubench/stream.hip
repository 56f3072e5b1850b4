// HBM streaming ceiling of one MI355X, measured with hand-written gfx950 streaming kernels (VERDICT r04
// Next #1).  tools/bw_probe.py measured torch's copy_ (5.0-5.4 TB/s beyond the Infinity Cache); this probe
// asks what a tuned streaming kernel reaches, so that the solve kernels' fractions can be stated against an
// achievable rate as well as against the 8 TB/s spec.
//
// Kernels (16 B per lane per access, every wave-instruction 1 KiB contiguous):
//   read   sum of a                        (bytes = |a|)
//   write  c = const                        (bytes = |c|)
//   copy   c = a                            (bytes = |a| + |c|)
//   solve  s' = s + (h, h), s twice the size of h: the fused ADMM row phase's mix
//          (s in 8 B/px, H^T y in 4 B/px, s out 8 B/px: 12 read : 8 written)
// Each in two access forms: `global_load/store_dwordx4` through a 64-bit pointer, and
// `buffer_load/store_dwordx4` through a buffer resource (the form the solve kernels use).  Workgroups stream
// tiles of 256*U float4, one contiguous run each ("chunked") or interleaved over the grid; U accesses per
// thread are issued before the first is used; cache-policy bits on the buffer forms (nt, sc0/sc1).
// Occupancy is set by the grid: WPC waves per CU over 256 CUs.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench/stream tools/ubench/stream.hip
// Run:   tools/ubench/stream [out.jsonl]      (one JSON line per configuration, best of 3 timings)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

using rsrc_t = __amdgpu_buffer_rsrc_t;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ inline rsrc_t mkr(const void* p, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
template <int AUX>
__device__ inline float4 bld(rsrc_t r, unsigned vo) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, vo, 0, AUX));
}
template <int AUX>
__device__ inline void bst(rsrc_t r, unsigned vo, float4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, vo, 0, AUX);
}

enum { READ = 0, WRITE = 1, COPY = 2, SOLVE = 3 };

// A tile = 256*U float4 of the primary array (SOLVE: 2*256*U of s and 256*U of h); the grid walks `tiles`
// tiles, either as one contiguous run per workgroup (IL = 0) or interleaved (IL = 1: tile b + i*grid).
// Every tile gets its own buffer resource (scalar work), so offsets stay within 32 bits at any size.
// AUXL / AUXS: cache-policy bits of the buffer loads / stores (gfx950: 1 = sc0, 2 = nt, 16 = sc1).
template <int MODE, int U, bool BUF, int IL, int AUXL, int AUXS>
__global__ __launch_bounds__(256) void stream_kernel(const float4* __restrict__ a, const float4* __restrict__ h,
                                                     float4* __restrict__ c, unsigned tiles, float* sink) {
    constexpr unsigned TS = 256 * U * (MODE == SOLVE ? 2 : 1);   // primary float4 per tile
    const unsigned per = tiles / gridDim.x;
    const unsigned t = threadIdx.x;
    float4 acc = {0.f, 0.f, 0.f, 0.f};
    for (unsigned k = 0; k < per; ++k) {
        const size_t tile = IL ? (size_t)k * gridDim.x + blockIdx.x : (size_t)blockIdx.x * per + k;
        const float4* ab = a + tile * TS;
        float4* cb = c + tile * TS;
        const float4* hb = h + tile * (TS / 2);
        rsrc_t ra = mkr(ab, TS * 16u), rc = mkr(cb, TS * 16u), rh = mkr(hb, TS * 8u);
        if constexpr (MODE == SOLVE) {
            // unit = 2 consecutive s float4 (a lane's (s1,s1',s2,s2') for 2 pixel pairs) + 1 h float4
            float4 s0[U], s1[U], hv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const unsigned i = u * 256 + t;
                if constexpr (BUF) {
                    s0[u] = bld<AUXL>(ra, (2 * i) * 16u); s1[u] = bld<AUXL>(ra, (2 * i + 1) * 16u);
                    hv[u] = bld<AUXL>(rh, i * 16u);
                } else {
                    s0[u] = ab[2 * i]; s1[u] = ab[2 * i + 1]; hv[u] = hb[i];
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const unsigned i = u * 256 + t;
                float4 o0 = {s0[u].x + hv[u].x, s0[u].y + hv[u].y, s0[u].z + hv[u].x, s0[u].w + hv[u].y};
                float4 o1 = {s1[u].x + hv[u].z, s1[u].y + hv[u].w, s1[u].z + hv[u].z, s1[u].w + hv[u].w};
                if constexpr (BUF) { bst<AUXS>(rc, (2 * i) * 16u, o0); bst<AUXS>(rc, (2 * i + 1) * 16u, o1); }
                else { cb[2 * i] = o0; cb[2 * i + 1] = o1; }
            }
        } else {
            float4 v[U];
            if constexpr (MODE != WRITE) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const unsigned i = u * 256 + t;
                    if constexpr (BUF) v[u] = bld<AUXL>(ra, i * 16u); else v[u] = ab[i];
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const unsigned i = u * 256 + t;
                if constexpr (MODE == READ) {
                    acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
                } else {
                    float4 o = MODE == WRITE ? make_float4((float)i, 1.f, 2.f, 3.f) : v[u];
                    if constexpr (BUF) bst<AUXS>(rc, i * 16u, o); else cb[i] = o;
                }
            }
        }
    }
    if (MODE == READ && acc.x + acc.y + acc.z + acc.w == -1.2345f) sink[t] = acc.x;   // keeps the loads live
}

template <int MODE, int U, bool BUF, int IL, int AUXL, int AUXS>
static float time_one(const float4* a, const float4* h, float4* c, unsigned tiles, int grid, float* sink, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto k = stream_kernel<MODE, U, BUF, IL, AUXL, AUXS>;
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, a, h, c, tiles, sink);
    CK(hipGetLastError());
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, a, h, c, tiles, sink);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms / reps < best) best = ms / reps;
    }
    CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
    return best;
}

static const char* kName[] = {"read", "write", "copy", "solve"};

template <int MODE, int U, bool BUF, int IL = 0, int AUXL = 0, int AUXS = 0>
static void run(FILE* out, const float4* a, const float4* h, float4* c, size_t ws_bytes, int wpc, float* sink,
                bool inplace = false) {
    // primary array size: read/write touch one array of ws; copy two of ws/2; solve s (ws*0.4) + s' (ws*0.4) +
    // h (ws*0.2): ws = 2|s| + |h| = 2.5|s|
    size_t prim = MODE == COPY ? ws_bytes / 2 : MODE == SOLVE ? ws_bytes * 2 / 5 : ws_bytes;
    const int grid = 256 * wpc / 4;                           // 256-thread workgroups = 4 waves each
    const size_t ts = (size_t)256 * U * (MODE == SOLVE ? 2 : 1);
    const unsigned tiles = (unsigned)(prim / 16 / ts / grid * grid);
    if (tiles == 0) return;   // working set smaller than one tile per workgroup
    const size_t n4 = tiles * ts;
    double bytes = MODE == READ || MODE == WRITE ? n4 * 16.0 : MODE == COPY ? n4 * 32.0 : n4 * 16.0 * 2.5;
    int reps = (int)(20e9 / bytes) + 2;
    float ms = time_one<MODE, U, BUF, IL, AUXL, AUXS>(a, h, inplace ? const_cast<float4*>(a) : c, tiles, grid, sink,
                                                     reps);
    double tbs = bytes / (ms * 1e-3) / 1e12;
    const char* acc = BUF ? "buffer_dwordx4" : "global_dwordx4";
    const char* lay = IL ? "interleaved" : "chunked";
    fprintf(out, "{\"kernel\": \"%s\", \"access\": \"%s\", \"layout\": \"%s\", \"aux_load\": %d, \"aux_store\": %d, "
                 "\"U\": %d, \"waves_per_cu\": %d, \"ws_bytes\": %zu, \"in_place\": %d, \"bytes\": %.0f, \"ms\": %.4f, "
                 "\"TBps\": %.3f}\n",
            kName[MODE], acc, lay, AUXL, AUXS, U, wpc, ws_bytes, (int)inplace, bytes, ms, tbs);
    fflush(out);
    printf("%-5s %-14s %-11s aux %d/%-2d U=%d wpc=%2d ws %6.0f MB%s %6.2f GB  %8.3f ms  %6.3f TB/s\n", kName[MODE], acc,
           lay, AUXL, AUXS, U, wpc, ws_bytes / 1048576.0, inplace ? " in place" : "", bytes / 1e9, ms, tbs);
    fflush(stdout);
}

template <int MODE, int U>
static void both(FILE* out, const float4* a, const float4* h, float4* c, size_t ws, int wpc, float* sink) {
    run<MODE, U, false>(out, a, h, c, ws, wpc, sink);
    run<MODE, U, true>(out, a, h, c, ws, wpc, sink);
}

// the access forms of one kernel at 4 GB, 16 waves per CU: layout and cache-policy bits
template <int MODE, int U>
static void forms(FILE* out, const float4* a, const float4* h, float4* c, float* sink) {
    const size_t ws = 4ull << 30;
    run<MODE, U, true, 1>(out, a, h, c, ws, 16, sink);
    run<MODE, U, false, 1>(out, a, h, c, ws, 16, sink);
    run<MODE, U, true, 0, 0, 2>(out, a, h, c, ws, 16, sink);     // nt stores
    run<MODE, U, true, 1, 0, 2>(out, a, h, c, ws, 16, sink);
    run<MODE, U, true, 0, 2, 2>(out, a, h, c, ws, 16, sink);     // nt loads and stores
    run<MODE, U, true, 0, 0, 16>(out, a, h, c, ws, 16, sink);    // sc1 stores
    run<MODE, U, true, 0, 0, 17>(out, a, h, c, ws, 16, sink);    // sc0 sc1 stores
}

int main(int argc, char** argv) {
    FILE* out = argc > 1 ? fopen(argv[1], "w") : stdout;
    if (!out) { perror("open"); return 1; }
    const bool cache_only = argc > 2 && argv[2][0] == 'c';   // section 4 only
    const size_t maxws = 8ull << 30;
    char *a, *c, *h;
    CK(hipMalloc(&a, maxws));
    CK(hipMalloc(&c, maxws));
    CK(hipMalloc(&h, maxws / 2));
    CK(hipMemset(a, 0, maxws)); CK(hipMemset(c, 0, maxws)); CK(hipMemset(h, 0, maxws / 2));
    float* sink;
    CK(hipMalloc(&sink, 4096));
    const float4* A = (const float4*)a;
    const float4* H = (const float4*)h;
    float4* C = (float4*)c;
    // 4) working sets around the 256 MiB Infinity Cache (the fused 256^2 solve holds 256 planes x 768 KiB = 192 MiB of
    //    s and H^T y per wave of workgroups, rewritten in place every iteration): the solve mix, to a second array
    //    and in place
    for (size_t mb : {64, 128, 192, 256, 384, 768}) {
        run<SOLVE, 4, true, 1>(out, A, H, C, mb << 20, 8, sink);
        run<SOLVE, 4, true, 1>(out, A, H, C, mb << 20, 8, sink, true);
        run<SOLVE, 2, true, 0>(out, A, H, C, mb << 20, 8, sink, true);
        run<COPY, 4, true, 0>(out, A, H, C, mb << 20, 8, sink);
    }
    if (cache_only) {
        if (out != stdout) fclose(out);
        return 0;
    }
    // 1) occupancy / unroll sweep at 4 GB
    for (int wpc : {8, 16, 32}) {
        both<READ, 4>(out, A, H, C, 4ull << 30, wpc, sink);
        both<WRITE, 4>(out, A, H, C, 4ull << 30, wpc, sink);
        both<COPY, 2>(out, A, H, C, 4ull << 30, wpc, sink);
        both<COPY, 4>(out, A, H, C, 4ull << 30, wpc, sink);
        both<SOLVE, 2>(out, A, H, C, 4ull << 30, wpc, sink);
    }
    both<READ, 8>(out, A, H, C, 4ull << 30, 16, sink);
    both<COPY, 8>(out, A, H, C, 4ull << 30, 16, sink);
    // 2) access forms for the mixed kernels
    forms<COPY, 4>(out, A, H, C, sink);
    forms<SOLVE, 2>(out, A, H, C, sink);
    forms<SOLVE, 4>(out, A, H, C, sink);
    forms<WRITE, 4>(out, A, H, C, sink);
    // 3) working-set sweep at 16 waves per CU (1 GB .. 8 GB, all beyond the 256 MiB Infinity Cache)
    for (size_t gb : {1, 2, 8}) {
        both<READ, 4>(out, A, H, C, gb << 30, 16, sink);
        both<WRITE, 4>(out, A, H, C, gb << 30, 16, sink);
        both<COPY, 4>(out, A, H, C, gb << 30, 16, sink);
        both<SOLVE, 2>(out, A, H, C, gb << 30, 16, sink);
    }
    CK(hipFree(a)); CK(hipFree(c)); CK(hipFree(h)); CK(hipFree(sink));
    if (out != stdout) fclose(out);
    return 0;
}
