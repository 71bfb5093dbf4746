// Stand-alone probe (not part of libflcodec): what one round of k_lone_resident's grid barrier
// costs on its own — G = 245 workgroups of 1024 threads (one per CU), the two-level arrival tree
// (4 groups), the last arriver reading the group replicas and releasing a 64-bit word that the
// others poll — with and without the agent-scope fences around the counters, with and without the
// histogram flush before the arrival (~890 non-returning atomics a workgroup into 4 replicas of
// 3 x 2048 bins, the speculative round's flush), and with the replicas read by the merger.
// Kernel time per launch (launches back to back) minus an empty launch of the same grid.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/probe_gridbar.hip -o tools/probe_gridbar
//   tools/probe_gridbar [G=245] [reps=200]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int NT = 1024, NG = 4, HB = 3 * 2048;
constexpr int C_GLOB = 0, C_GEN = 32, C_GRP = 128, C_REP = 1024, C_SIZE = C_REP + NG * HB;

template <int FENCE, int FLUSH, int MERGE>
__global__ __launch_bounds__(NT) void k_bar(uint32_t* ctl, uint32_t* sink) {
    __shared__ uint32_t flag_s, gen_s, acc_s;
    const uint32_t G = gridDim.x, g = blockIdx.x, t = threadIdx.x;
    const uint32_t grp = g % NG, ngr = min(G, (uint32_t)NG), gsz = (G - grp + NG - 1) / NG;
    uint64_t* gw = reinterpret_cast<uint64_t*>(ctl + C_GEN);
    if (t == 0) gen_s = (uint32_t)__hip_atomic_load(gw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 7u;
    if (FLUSH && t < 890) {
        const uint32_t bin = (g * 7919u + t * 13u) % HB;
        __hip_atomic_fetch_add(ctl + C_REP + grp * HB + bin, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
        uint32_t last = 0;
        if (FENCE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        uint32_t* gc = ctl + C_GRP + 32 * grp;
        if (__hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsz - 1u) {
            if (FENCE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (FENCE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            if (__hip_atomic_fetch_add(ctl + C_GLOB, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ngr - 1u) {
                __hip_atomic_store(ctl + C_GLOB, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (FENCE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                last = 1;
            }
        }
        flag_s = last;
        acc_s = 0;
    }
    __syncthreads();
    if (flag_s) {
        uint32_t c = 0;
        if (MERGE)
            for (int i = t; i < HB; i += NT)
#pragma unroll
                for (int r = 0; r < NG; ++r) {
                    c += __hip_atomic_load(ctl + C_REP + r * HB + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(ctl + C_REP + r * HB + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
        if (c) atomicAdd(&acc_s, c);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) {
            if (FENCE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            __hip_atomic_store(gw, (uint64_t)((gen_s + 1u) & 7u) | ((uint64_t)acc_s << 3), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    } else if (t == 0) {
        const uint64_t t0 = wall_clock64();
        for (;;) {
            const uint64_t w = __hip_atomic_load(gw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (((uint32_t)w & 7u) != gen_s) break;
            __builtin_amdgcn_s_sleep(1);
            if (wall_clock64() - t0 > 10000000ull) { sink[1] = 1; break; }   // 0.1 s: give up (probe)
        }
        if (FENCE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
}

__global__ __launch_bounds__(NT) void k_empty(uint32_t* sink) {
    if (threadIdx.x == 1023 && blockIdx.x == 100000) sink[0] = 1;
}

int main(int argc, char** argv) {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int G = argc > 1 ? atoi(argv[1]) : 245;
    const int reps = argc > 2 ? atoi(argv[2]) : 200;
    if (G > cus) { printf("G > CUs: not co-resident\n"); return 1; }
    uint32_t *ctl, *sink;
    CK(hipMalloc(&ctl, C_SIZE * 4));
    CK(hipMemset(ctl, 0, C_SIZE * 4));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(sink, 0, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, auto launch) {
        for (int i = 0; i < 10; ++i) launch();
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < 3; ++r) {
            CK(hipEventRecord(e0, 0));
            for (int k = 0; k < reps; ++k) launch();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        uint32_t s[2];
        CK(hipMemcpy(s, sink, 8, hipMemcpyDeviceToHost));
        printf("{\"kernel\": \"%s\", \"G\": %d, \"us_per_launch\": %.2f, \"gave_up\": %u}\n", name, G, best * 1e3 / reps, s[1]);
        fflush(stdout);
    };
    timeit("empty", [&] { hipLaunchKernelGGL(k_empty, dim3(G), dim3(NT), 0, 0, sink); });
    timeit("bar_nofence", [&] { hipLaunchKernelGGL((k_bar<0, 0, 0>), dim3(G), dim3(NT), 0, 0, ctl, sink); });
    timeit("bar_fence", [&] { hipLaunchKernelGGL((k_bar<1, 0, 0>), dim3(G), dim3(NT), 0, 0, ctl, sink); });
    timeit("bar_fence_merge", [&] { hipLaunchKernelGGL((k_bar<1, 0, 1>), dim3(G), dim3(NT), 0, 0, ctl, sink); });
    timeit("bar_fence_flush_merge", [&] { hipLaunchKernelGGL((k_bar<1, 1, 1>), dim3(G), dim3(NT), 0, 0, ctl, sink); });
    timeit("bar_nofence_flush_merge", [&] { hipLaunchKernelGGL((k_bar<0, 1, 1>), dim3(G), dim3(NT), 0, 0, ctl, sink); });
    return 0;
}
