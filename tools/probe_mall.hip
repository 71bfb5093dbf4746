// Stand-alone probe (not part of libflcodec): can a persistent, one-workgroup-per-CU kernel read
// each client row from HBM once for its norm and re-read it for the encode from the 256 MiB
// Infinity Cache one step later?  Times the access patterns of the candidate QSGD designs over a
// [N, D] fp32 matrix (sums only, no codec work).
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/probe_mall.hip -o tools/probe_mall
//   tools/probe_mall [N] [D]
//
// modes:  stream     grid-stride read of the whole matrix (baseline, 4ND bytes)
//         twopass    stream twice (the current norm pass + encode pass)
//         pers1      persistent: WG w reads its column slice of row 0..N-1 in order (4ND)
//         lag        persistent: step i reads row i+1's slice, then row i's slice again (8ND)
//         lagsync    lag + the per-row cross-workgroup hand-off (partials + counter)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int TPB = 512;
constexpr int UNR = 8;

__global__ void k_fill(float* x, int64_t total) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
        x[i] = (float)((i * 2654435761u) & 0xFFFF) * 1e-4f - 3.f;
}

__global__ __launch_bounds__(256) void k_stream(const float4* x, int64_t groups, float* out) {
    float a = 0.f;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; g + (UNR - 1) * stride < groups; g += UNR * stride) {
        float4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) v[u] = x[g + u * stride];
#pragma unroll
        for (int u = 0; u < UNR; ++u) a += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    for (; g < groups; g += stride) { float4 v = x[g]; a += v.x + v.y + v.z + v.w; }
    if (a == 12345.f) out[0] = a;
}

// sum of one workgroup's slice [s0, s1) (float4 groups) of one row
__device__ inline float slice_sum(const float4* r, int64_t s0, int64_t s1) {
    float a = 0.f;
    int64_t g = s0 + threadIdx.x;
    for (; g + (UNR - 1) * TPB < s1; g += UNR * TPB) {
        float4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) v[u] = r[g + u * TPB];
#pragma unroll
        for (int u = 0; u < UNR; ++u) a += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    for (; g < s1; g += TPB) { float4 v = r[g]; a += v.x + v.y + v.z + v.w; }
    return a;
}

__device__ inline float block_sum(float a, float* red) {
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
    __syncthreads();
    float t = 0.f;
    for (int w = 0; w < TPB / 64; ++w) t += red[w];
    __syncthreads();
    return t;
}

template <int MODE>   // 0 pers1, 1 lag, 2 lagsync
__global__ __launch_bounds__(TPB) void k_pers(const float4* x, int64_t n, int64_t dg, int64_t per_wg,
                                              double* partial, uint32_t* cnt, float* out, uint32_t* timeout) {
    __shared__ float red[TPB / 64];
    __shared__ float nrm;
    const int G = gridDim.x, w = blockIdx.x;
    const int64_t s0 = (int64_t)w * per_wg, s1 = min(dg, s0 + per_wg);
    float acc = 0.f;
    if (MODE == 0) {
        for (int64_t i = 0; i < n; ++i) acc += slice_sum(x + i * dg, s0, s1);
    } else {
        // prologue: row 0's partial
        float p = block_sum(slice_sum(x, s0, s1), red);
        if (MODE == 2 && threadIdx.x == 0) {
            __hip_atomic_store(&partial[w], (double)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_fetch_add(&cnt[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        for (int64_t i = 0; i < n; ++i) {
            if (i + 1 < n) {
                p = block_sum(slice_sum(x + (i + 1) * dg, s0, s1), red);
                if (MODE == 2 && threadIdx.x == 0) {
                    __hip_atomic_store(&partial[(i + 1) * G + w], (double)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __hip_atomic_fetch_add(&cnt[(i + 1) * 32], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            if (MODE == 2) {
                if (threadIdx.x < 64) {
                    if (threadIdx.x == 0) {
                        uint32_t spins = 0;
                        while (__hip_atomic_load(&cnt[i * 32], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (uint32_t)G) {
                            __builtin_amdgcn_s_sleep(2);
                            if (++spins > (1u << 24)) { atomicOr(timeout, 1u); break; }
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                    double s = 0.0;
                    for (int k = threadIdx.x; k < G; k += 64)
                        s += __hip_atomic_load(&partial[i * G + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
                    if (threadIdx.x == 0) nrm = (float)s;
                }
                __syncthreads();
                acc += nrm * 1e-30f;
            }
            acc += slice_sum(x + i * dg, s0, s1);
        }
    }
    if (acc == 12345.f) out[0] = acc;
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 64;
    const int64_t d = argc > 2 ? atoll(argv[2]) : 25000000;
    const int64_t dg = d / 4;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int G = prop.multiProcessorCount;
    printf("CUs %d  N %lld  D %lld  matrix %.2f GB\n", G, (long long)n, (long long)d, 4.0 * n * d / 1e9);
    float4* x;
    CK(hipMalloc(&x, (size_t)n * dg * 16));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, (float*)x, n * dg * 4);
    double* partial;
    uint32_t *cnt, *timeout;
    float* out;
    CK(hipMalloc(&partial, (size_t)n * G * 8));
    CK(hipMalloc(&cnt, (size_t)n * 32 * 4));
    CK(hipMalloc(&timeout, 4));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(timeout, 0, 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int64_t per_wg = (dg + G - 1) / G;
    const double bytes = 4.0 * n * d;
    auto run = [&](const char* name, int mode, int reps) {
        float best = 1e30f;
        for (int r = 0; r < reps; ++r) {
            CK(hipMemset(cnt, 0, (size_t)n * 32 * 4));
            CK(hipEventRecord(e0));
            if (mode == 10) {
                hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, x, n * dg, out);
            } else if (mode == 11) {
                hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, x, n * dg, out);
                hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, x, n * dg, out);
            } else {
                void* args[] = {&x, (void*)&n, (void*)&dg, (void*)&per_wg, &partial, &cnt, &out, &timeout};
                const void* fn = mode == 0 ? (const void*)k_pers<0> : mode == 1 ? (const void*)k_pers<1> : (const void*)k_pers<2>;
                CK(hipLaunchCooperativeKernel(fn, dim3(G), dim3(TPB), args, 0, 0));
            }
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        uint32_t to = 0;
        CK(hipMemcpy(&to, timeout, 4, hipMemcpyDeviceToHost));
        printf("%-9s %9.3f ms   %7.0f GB/s of 4ND (algorithmic)%s\n", name, best, bytes / best / 1e6, to ? "  TIMEOUT" : "");
    };
    run("stream", 10, 3);
    run("twopass", 11, 3);
    run("pers1", 0, 3);
    run("lag", 1, 3);
    run("lagsync", 2, 3);
    return 0;
}
