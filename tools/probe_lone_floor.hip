// Stand-alone probe (not part of libflcodec): the floor of a lone compressVector row at D = 10 M
// (the drop-in TopK call, k_lone_resident's layout) without any selection work — what one launch
// that reads x and writes the dense [D] output costs, in the resident layout (one 1024-thread
// workgroup per CU, e4 float4 a thread in registers) and in an occupancy-rich one.  Rows rotate
// over N = 32 clients like bench.py --dropin; the threshold is a fixed |x| > 2.576 (1 % of a
// Gaussian row), so the stores have the real output's zero / nonzero mix.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/probe_lone_floor.hip -o tools/probe_lone_floor
//   tools/probe_lone_floor [D=10000000] [N=32] [reps=20] [contiguous=0|1]
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int NT = 1024, RU = 16;
typedef unsigned int u4v __attribute__((ext_vector_type(4)));

__global__ void k_fill(float* x, int64_t total, uint32_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        // sum of 4 uniforms, scaled: roughly Gaussian (the threshold keeps ~1-2 %)
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        float s = 0.f;
        for (int k = 0; k < 4; ++k) { h = h * 1664525u + 1013904223u; s += (float)(h >> 8) * (1.f / 16777216.f); }
        x[i] = (s - 2.f) * 1.732f;
    }
}

__device__ inline uint32_t thr_keep(uint32_t b) { return (b & 0x7FFFFFFFu) > 0x4024DD2Fu ? b : 0u; }   // |x| > 2.576

// the resident layout: G workgroups of 1024 threads, e4 float4 a thread (loads all issued first)
// GEN: 0 none, 1 every thread loads a shared control word (agent-scope atomic) before the row,
// 2 only thread 0 does
template <bool STORE, int GEN = 0>
__global__ __launch_bounds__(NT) void k_res(const float* x, int64_t d, int e4, float* out, uint32_t* sink, uint32_t delay = 0) {
    const uint32_t g = blockIdx.x, t = threadIdx.x;
    uint64_t gw = 0;
    if (GEN == 1 || (GEN == 2 && t == 0))
        gw = __hip_atomic_load(reinterpret_cast<const uint64_t*>(sink + 8), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int64_t gb = (int64_t)g * e4 * NT * 4;
    const auto rxg = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x) + gb, (short)0,
                                                       (int)(min((int64_t)e4 * NT * 4, d - gb) * 4), 0x00020000);
    const auto rog = __builtin_amdgcn_make_buffer_rsrc(out + gb, (short)0, (int)(min((int64_t)e4 * NT * 4, d - gb) * 4), 0x00020000);
    u4v v[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rxg, t * 16u, u * NT * 16, 2);
    if (STORE && delay) {             // a pause between the loads landing and the stores (the selection's rounds)
        uint32_t a = 0;
#pragma unroll
        for (int u = 0; u < RU; ++u) a |= v[u][0];
        if (a == 0x7FFFFFFFu) sink[2] = a;                 // (waits for the loads)
        const uint64_t t0 = wall_clock64();
        while (wall_clock64() - t0 < delay) __builtin_amdgcn_s_sleep(2);
    }
    if (STORE) {
#pragma unroll
        for (int u = 0; u < RU; ++u) {
            if (u < e4) {
                const u4v o = {thr_keep(v[u][0]), thr_keep(v[u][1]), thr_keep(v[u][2]), thr_keep(v[u][3])};
                __builtin_amdgcn_raw_buffer_store_b128(o, rog, t * 16u, u * NT * 16, 2);
            }
        }
    } else {
        uint32_t a = 0;
#pragma unroll
        for (int u = 0; u < RU; ++u) a += v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
        if (a + (uint32_t)gw == 0x12345u) sink[0] = a;
    }
}

// occupancy-rich: 256-thread workgroups, 4 float4 a thread
__global__ __launch_bounds__(256) void k_wide(const float* x, int64_t d, float* out) {
    const int64_t d4 = (d + 3) / 4;
    const int64_t b = (int64_t)blockIdx.x * 1024;
    const auto rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x) + 4 * b, (short)0, (int)(min((int64_t)4096, d - 4 * b) * 4), 0x00020000);
    const auto ro = __builtin_amdgcn_make_buffer_rsrc(out + 4 * b, (short)0, (int)(min((int64_t)4096, d - 4 * b) * 4), 0x00020000);
    (void)d4;
    u4v v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rx, threadIdx.x * 16u, u * 4096, 2);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const u4v o = {thr_keep(v[u][0]), thr_keep(v[u][1]), thr_keep(v[u][2]), thr_keep(v[u][3])};
        __builtin_amdgcn_raw_buffer_store_b128(o, ro, threadIdx.x * 16u, u * 4096, 2);
    }
}

__global__ __launch_bounds__(NT) void k_empty(uint32_t* sink) {
    if (threadIdx.x == 1023 && blockIdx.x == 100000) sink[0] = 1;
}

int main(int argc, char** argv) {
    const int64_t d = argc > 1 ? atoll(argv[1]) : 10000000;
    const int n = argc > 2 ? atoi(argv[2]) : 32;
    const int reps = argc > 3 ? atoi(argv[3]) : 20;
    const int contiguous = argc > 4 ? atoi(argv[4]) : 0;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    float *x, *out;
    uint32_t* sink;
    const size_t xb = (size_t)n * d * 4;
    if (contiguous) CK(hipExtMallocWithFlags((void**)&x, xb, hipDeviceMallocContiguous));
    else CK(hipMalloc(&x, xb));
    CK(hipMalloc(&out, (size_t)d * 4));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(sink, 0, 64));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, x, (int64_t)n * d, 7u);
    CK(hipDeviceSynchronize());
    const int64_t d4 = (d + 3) / 4;
    // k_lone_resident's grid: the fewest float4 a thread that fits one workgroup per CU
    int e4 = (int)((d4 + (int64_t)cus * NT - 1) / ((int64_t)cus * NT));
    const int G = (int)((d4 + (int64_t)e4 * NT - 1) / ((int64_t)e4 * NT));
    if (e4 > RU) { printf("row too long for the resident layout\n"); return 1; }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, auto launch) {
        for (int i = 0; i < n; ++i) launch(x + (size_t)i * d);
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < 3; ++r) {
            CK(hipEventRecord(e0, 0));
            for (int k = 0; k < reps; ++k)
                for (int i = 0; i < n; ++i) launch(x + (size_t)i * d);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        const double us = best * 1e3 / (reps * n);
        printf("{\"kernel\": \"%s\", \"d\": %lld, \"contiguous\": %d, \"G\": %d, \"e4\": %d, \"us_per_call\": %.2f, \"GBps_8D\": %.0f}\n",
               name, (long long)d, contiguous, G, e4, us, 8.0 * d / (us * 1e3));
        fflush(stdout);
    };
    timeit("empty_G_1024", [&](const float*) { hipLaunchKernelGGL(k_empty, dim3(G), dim3(NT), 0, 0, sink); });
    timeit("res_load_only", [&](const float* r) { hipLaunchKernelGGL(k_res<false>, dim3(G), dim3(NT), 0, 0, r, d, e4, out, sink); });
    timeit("res_load_only_gen_all", [&](const float* r) { hipLaunchKernelGGL((k_res<false, 1>), dim3(G), dim3(NT), 0, 0, r, d, e4, out, sink); });
    timeit("res_load_only_gen_t0", [&](const float* r) { hipLaunchKernelGGL((k_res<false, 2>), dim3(G), dim3(NT), 0, 0, r, d, e4, out, sink); });
    timeit("res_load_store", [&](const float* r) { hipLaunchKernelGGL(k_res<true>, dim3(G), dim3(NT), 0, 0, r, d, e4, out, sink); });
    for (uint32_t dl : {500u, 1000u, 2000u})
        timeit(dl == 500u ? "res_load_5us_store" : dl == 1000u ? "res_load_10us_store" : "res_load_20us_store",
               [&](const float* r) { hipLaunchKernelGGL((k_res<true>), dim3(G), dim3(NT), 0, 0, r, d, e4, out, sink, dl); });
    timeit("empty_5us", [&](const float* r) { hipLaunchKernelGGL((k_res<true>), dim3(G), dim3(NT), 0, 0, r, 0, e4, out, sink, 500u); });
    timeit("wide_load_store", [&](const float* r) { hipLaunchKernelGGL(k_wide, dim3((unsigned)((d4 + 1023) / 1024)), dim3(256), 0, 0, r, d, out); });
    return 0;
}
