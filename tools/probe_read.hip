// Stand-alone probe (not part of libflcodec): the HBM read ceiling of the C4 shard's access
// pattern in three load forms, over the same [N, D] fp32 allocation.  Sums only, no codec work.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/probe_read.hip -o tools/probe_read
//   tools/probe_read [N=512] [D=25000000] [reps=5]
//
// modes:  reg    grid-stride float4 nontemporal loads, 8 per lane in flight (the fold's pattern)
//         ring   the sparse filters' item walk: items of 8192 elements of one row, blocks of 16
//                rows with the row fastest, a RING-deep register ring of nt buffer loads
//         glds   the same item walk, but the row bytes go HBM -> LDS by LDS-DMA
//                (buffer_load_dwordx4 ... lds nt), A pieces of 1 KiB ahead per wave, consumed by
//                ds_read_b128 from a per-wave ring
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int CHUNK = 4096, FGS = 2, RB = 16;

__global__ void k_fill(float* x, int64_t total) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
        x[i] = (float)((i * 2654435761u) & 0xFFFF) * 1e-4f - 3.f;
}

__global__ __launch_bounds__(256) void k_reg(const float4* x, int64_t groups, float* out) {
    typedef float v4f __attribute__((ext_vector_type(4)));
    float a = 0.f;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; g + 7 * stride < groups; g += 8 * stride) {
        v4f v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(x + g + u * stride));
#pragma unroll
        for (int u = 0; u < 8; ++u) a += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    for (; g < groups; g += stride) { float4 v = x[g]; a += v.x + v.y + v.z + v.w; }
    if (a == 12345.f) out[0] = a;
}

__device__ inline void item_at(int64_t t, int64_t rn, int64_t G, int64_t& r, int64_t& g) {
    const int64_t blk = t / (RB * G), rem = t - blk * RB * G;
    const int64_t bn = min((int64_t)RB, rn - blk * RB);
    g = rem / bn;
    r = blk * RB + (rem - g * bn);
}
__device__ inline __amdgpu_buffer_rsrc_t rsrc_of(const float* x, int64_t d, int64_t r, int64_t j0) {
    const int64_t len = max((int64_t)0, min((int64_t)(FGS * CHUNK), d - j0));
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x + r * d + j0), (short)0, (int)(len * 4), 0x00020000);
}

// ring: one wave per item, 32 loads of 1 KiB per item, RING deep across items
template <int RING>
__global__ __launch_bounds__(256) void k_ring(const float* x, int64_t n, int64_t d, float* out) {
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t G = (d + FGS * CHUNK - 1) / (FGS * CHUNK);
    const int64_t items = n * G, stride = (int64_t)gridDim.x * 4;
    int64_t it = (int64_t)blockIdx.x * 4 + wv;
    if (it >= items) return;
    int64_t r, g;
    item_at(it, n, G, r, g);
    auto rs = rsrc_of(x, d, r, g * FGS * CHUNK);
    float4 ring[RING];
    auto ld = [&](__amdgpu_buffer_rsrc_t q, int L) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(q, lane * 16, L * 1024, 2);
        return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
    };
#pragma unroll
    for (int L = 0; L < RING - 1; ++L) ring[L] = ld(rs, L);
    float a = 0.f;
    while (it < items) {
        const int64_t nit = it + stride;
        __amdgpu_buffer_rsrc_t rsn;
        if (nit < items) { int64_t nr, ng; item_at(nit, n, G, nr, ng); rsn = rsrc_of(x, d, nr, ng * FGS * CHUNK); }
        else rsn = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), (short)0, 0, 0x00020000);
#pragma unroll
        for (int L = 0; L < 32; ++L) {
            const int P = L + RING - 1;
            ring[P % RING] = P < 32 ? ld(rs, P) : ld(rsn, P - 32);
            const float4 v = ring[L % RING];
            a += (v.x + v.y) + (v.z + v.w);
        }
        rs = rsn;
        it = nit;
    }
    if (a == 12345.f) out[0] = a;
}

// glds: one wave per item; pieces of 1 KiB go HBM -> LDS, A ahead, ring of S slots per wave
template <int A, int S>
__global__ __launch_bounds__(256) void k_glds(const float* x, int64_t n, int64_t d, float* out) {
    __shared__ __attribute__((aligned(16))) float4 lds[4][S][64];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t G = (d + FGS * CHUNK - 1) / (FGS * CHUNK);
    const int64_t items = n * G, stride = (int64_t)gridDim.x * 4;
    int64_t it = (int64_t)blockIdx.x * 4 + wv;
    if (it >= items) return;
    int64_t r, g;
    item_at(it, n, G, r, g);
    auto rs = rsrc_of(x, d, r, g * FGS * CHUNK);
    __amdgpu_buffer_rsrc_t rsn = rs;
    bool have_next = false;
    auto issue = [&](__amdgpu_buffer_rsrc_t q, int L, int slot) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(q, (__attribute__((address_space(3))) void*)&lds[wv][slot][0], 16, lane * 16,
                                                 L * 1024, 0, 2);
    };
    // pieces are numbered globally per wave: piece k = item k / 32, piece L = k % 32
#pragma unroll
    for (int k = 0; k < A; ++k) issue(rs, k, k % S);
    float a = 0.f;
    int64_t k = 0;
    while (it < items) {
        const int64_t nit = it + stride;
        if (nit < items) { int64_t nr, ng; item_at(nit, n, G, nr, ng); rsn = rsrc_of(x, d, nr, ng * FGS * CHUNK); }
        else rsn = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), (short)0, 0, 0x00020000);
        (void)have_next;
#pragma unroll
        for (int L = 0; L < 32; ++L, ++k) {
            const int P = L + A;
            const int slot = (int)((k + A) % S);
            if (P < 32) issue(rs, P, slot); else issue(rsn, P - 32, slot);
            // wait for piece k (A newer pieces may stay in flight), then read it; both in asm so
            // that hipcc adds no vmcnt(0) of its own for the LDS alias
            typedef float v4f __attribute__((ext_vector_type(4)));
            v4f v;
            const uint32_t la = (uint32_t)(size_t)(__attribute__((address_space(3))) float4*)&lds[wv][k % S][lane];
            asm volatile("s_waitcnt vmcnt(%1)\n\tds_read_b128 %0, %2\n\ts_waitcnt lgkmcnt(0)" : "=&v"(v) : "n"(A), "v"(la) : "memory");
            a += (v.x + v.y) + (v.z + v.w);
        }
        rs = rsn;
        it = nit;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (a == 12345.f) out[0] = a;
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 512, d = argc > 2 ? atoll(argv[2]) : 25000000;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    const int allocs = argc > 4 ? atoi(argv[4]) : 2;
    const double bytes = 4.0 * n * d;
    float* out;
    CK(hipMalloc(&out, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int64_t G = (d + FGS * CHUNK - 1) / (FGS * CHUNK);
    const int gw = (int)std::min<int64_t>((n * G + 3) / 4, 32768);
    for (int al = 0; al < allocs; ++al) {
        float* x;
        CK(hipMalloc(&x, (size_t)(4 * n * d)));
        hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, x, n * d);
        CK(hipDeviceSynchronize());
        auto timeit = [&](const char* name, auto launch) {
            launch();
            CK(hipDeviceSynchronize());
            float best = 1e30f, sum = 0.f;
            for (int r = 0; r < reps; ++r) {
                CK(hipEventRecord(e0, 0));
                launch();
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = ms < best ? ms : best;
                sum += ms;
            }
            printf("alloc %d %-22s best %8.3f ms  mean %8.3f ms  %6.3f TB/s (best)\n", al, name, best, sum / reps,
                   bytes / best * 1e-9);
            fflush(stdout);
        };
        timeit("reg g=cus*8", [&] { hipLaunchKernelGGL(k_reg, dim3(cus * 8), dim3(256), 0, 0, (const float4*)x, n * d / 4, out); });
        timeit("reg g=cus*32", [&] { hipLaunchKernelGGL(k_reg, dim3(cus * 32), dim3(256), 0, 0, (const float4*)x, n * d / 4, out); });
        timeit("ring16", [&] { hipLaunchKernelGGL(k_ring<16>, dim3(gw), dim3(256), 0, 0, x, n, d, out); });
        timeit("ring8", [&] { hipLaunchKernelGGL(k_ring<8>, dim3(gw), dim3(256), 0, 0, x, n, d, out); });
        timeit("glds A8 S10", [&] { hipLaunchKernelGGL((k_glds<8, 10>), dim3(gw), dim3(256), 0, 0, x, n, d, out); });
        timeit("glds A16 S18", [&] { hipLaunchKernelGGL((k_glds<16, 18>), dim3(gw), dim3(256), 0, 0, x, n, d, out); });
        timeit("glds A24 S26", [&] { hipLaunchKernelGGL((k_glds<24, 26>), dim3(gw), dim3(256), 0, 0, x, n, d, out); });
        timeit("ring16 grid=res", [&] { hipLaunchKernelGGL(k_ring<16>, dim3(cus * 8), dim3(256), 0, 0, x, n, d, out); });
        timeit("glds A16 grid=res", [&] { hipLaunchKernelGGL((k_glds<16, 18>), dim3(cus * 2), dim3(256), 0, 0, x, n, d, out); });
        CK(hipFree(x));
    }
    return 0;
}
