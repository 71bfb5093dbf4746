// Stand-alone probe (not part of libflcodec): the C4 fold's list walk (k_ds_accum) without its
// arithmetic, to tell the access pattern's own cost from the kernel's.  One 64-lane workgroup per
// half-chunk tile (H = 12207 at D = 25 M) with an 8 KB LDS tile (the fold's occupancy), walking
// n = 256 rows with a 16-row register ring; loads are summed, nothing else.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/probe_walk.hip -o tools/probe_walk
//   tools/probe_walk [H=12207] [n=256] [reps=5]
//
// modes:  fixed   the product layout: row r of tile h at (h n + r) 256 B, the first 128 B read
//                 (64 u16 entries, one per lane)
//         packed  the same entries with the rows of a tile contiguous at 96 B each (48 entries:
//                 the C4 lists hold ~41), lanes >= 48 idle
//         lds     fixed, plus the fold's per-row LDS read-modify-write of the tile (64 distinct
//                 columns per row, rows in order)
//         meta    lds, plus the fold's per-batch row state: a u32 per row loaded one 64-row batch
//                 ahead, whose value (readlane) picks each refill's address (k_ds_accum's cnt)
//         ldsrand lds with each row's 64 distinct columns at random banks (lane * 32 + a hash < 32)
//         dense   each wave streams its tile's whole 64 KB region with 16-B-per-lane loads
//                 (1 KB per load, 16 in flight): the bytes-in-flight bound of the same footprint
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int AP = 16;
__device__ inline uint32_t hmix(uint32_t v) {
    v *= 2654435761u; v ^= v >> 16; v *= 0x85EBCA6Bu; v ^= v >> 13; v *= 0xC2B2AE35u; v ^= v >> 16;
    return v;
}

template <int MODE>
__global__ __launch_bounds__(64) void k_walk(const uint8_t* __restrict__ base, int64_t H, int64_t n, uint32_t* out,
                                             const uint32_t* __restrict__ mbase) {
    extern __shared__ float tile[];
    const int lane = threadIdx.x;
    const int64_t h = blockIdx.x;
    if (h >= H) return;
    for (int i = lane; i < 2048; i += 64) tile[i] = 0.f;
    uint32_t acc = 0;
    if (MODE == 4) {
        const uint32_t* meta = mbase + h * n;
        const uint16_t* p = reinterpret_cast<const uint16_t*>(base + h * n * 256);
        uint32_t cur = meta[lane], nxt = 0;
        uint32_t r[AP];
#pragma unroll
        for (int u = 0; u < AP; ++u) {
            const uint32_t c = __builtin_amdgcn_readlane(cur, u);
            r[u] = p[(c ? u : 0) * 128 + lane];
        }
        for (int64_t b = 0; b < n / 64; ++b) {
            nxt = (b + 1) * 64 + lane < n ? meta[(b + 1) * 64 + lane] : 0u;
#pragma unroll
            for (int q = 0; q < 64; ++q) {
                const int u = q % AP;
                acc += r[u];
                const uint32_t loc = ((uint32_t)lane * 37u + (uint32_t)q * 11u + r[u]) & 2047u;
                tile[loc] = tile[loc] + 1.0f;
                const int nq = q + AP;
                const uint32_t c = nq < 64 ? __builtin_amdgcn_readlane(cur, nq) : __builtin_amdgcn_readlane(nxt, nq - 64);
                const int64_t row = b * 64 + nq;
                r[u] = (row < n && c) ? (uint32_t)p[row * 128 + lane] : 0u;
            }
            cur = nxt;
        }
    } else if (MODE == 2) {
        const uint4* p = reinterpret_cast<const uint4*>(base + h * n * 256);
        const int64_t nl = n * 256 / 1024;             // 1 KB per wave load
        uint4 r[AP];
#pragma unroll
        for (int u = 0; u < AP; ++u) r[u] = u < nl ? p[u * 64 + lane] : make_uint4(0, 0, 0, 0);
        for (int64_t q = 0; q < nl; q += AP) {
#pragma unroll
            for (int u = 0; u < AP; ++u) {
                acc += r[u].x ^ r[u].y ^ r[u].z ^ r[u].w;
                const int64_t nq = q + AP + u;
                r[u] = nq < nl ? p[nq * 64 + lane] : make_uint4(0, 0, 0, 0);
            }
        }
    } else {
        const int64_t rs = MODE != 1 ? 256 : 96;   // (modes 0, 3, 5: the product layout)       // bytes per row region
        const int ne = MODE != 1 ? 64 : 48;
        const uint16_t* p = reinterpret_cast<const uint16_t*>(base + (MODE != 1 ? h * n * 256 : h * n * 96));
        uint32_t r[AP];
#pragma unroll
        for (int u = 0; u < AP; ++u) r[u] = lane < ne ? p[u * (rs / 2) + lane] : 0u;
        for (int64_t q = 0; q < n; q += AP) {
#pragma unroll
            for (int u = 0; u < AP; ++u) {
                acc += r[u];
                if (MODE == 3 || MODE == 5) {
                    // 3: 64 distinct banks per row; 5: hashed columns (distinct, random banks, as real lists)
                    const uint32_t loc = MODE == 3 ? (((uint32_t)lane * 37u + (uint32_t)(q + u) * 11u + r[u]) & 2047u)
                                                   : (((uint32_t)lane * 32u + (hmix((uint32_t)(q + u) * 64u + (uint32_t)lane) >> 27)) & 2047u);
                    tile[loc] = tile[loc] + 1.0f;
                }
                const int64_t nq = q + AP + u;
                r[u] = (nq < n && lane < ne) ? p[nq * (rs / 2) + lane] : 0u;
            }
        }
    }
    tile[lane] += (float)acc;
    if (tile[lane] == 1234.5f) out[h] = acc;
}

int main(int argc, char** argv) {
    const int64_t H = argc > 1 ? atoll(argv[1]) : 12207, n = argc > 2 ? atoll(argv[2]) : 256;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    const size_t bytes = (size_t)H * n * 256;
    uint8_t* base;
    uint32_t* out;
    CK(hipMalloc(&base, bytes));
    CK(hipMalloc(&out, H * 4));
    CK(hipMemset(base, 1, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    uint32_t* meta;
    CK(hipMalloc(&meta, (size_t)H * n * 4));
    CK(hipMemset(meta, 1, (size_t)H * n * 4));
    const char* names[6] = {"fixed", "packed", "dense", "lds", "meta", "ldsrand"};
    const double moved[6] = {(double)H * n * 128, (double)H * n * 96, (double)H * n * 256, (double)H * n * 128, (double)H * n * 128, (double)H * n * 128};
    for (int rep = 0; rep < reps; ++rep) {
        for (int m = 0; m < 6; ++m) {
            CK(hipEventRecord(e0, 0));
            if (m == 0) hipLaunchKernelGGL(k_walk<0>, dim3((unsigned)H), dim3(64), 8192, 0, base, H, n, out, meta);
            if (m == 1) hipLaunchKernelGGL(k_walk<1>, dim3((unsigned)H), dim3(64), 8192, 0, base, H, n, out, meta);
            if (m == 2) hipLaunchKernelGGL(k_walk<2>, dim3((unsigned)H), dim3(64), 8192, 0, base, H, n, out, meta);
            if (m == 3) hipLaunchKernelGGL(k_walk<3>, dim3((unsigned)H), dim3(64), 8192, 0, base, H, n, out, meta);
            if (m == 4) hipLaunchKernelGGL(k_walk<4>, dim3((unsigned)H), dim3(64), 8192, 0, base, H, n, out, meta);
            if (m == 5) hipLaunchKernelGGL(k_walk<5>, dim3((unsigned)H), dim3(64), 8192, 0, base, H, n, out, meta);
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("{\"rep\": %d, \"mode\": \"%s\", \"us\": %.1f, \"GBps_read\": %.0f}\n", rep, names[m], ms * 1e3,
                   moved[m] / (ms * 1e-3) / 1e9);
        }
    }
    CK(hipFree(base));
    CK(hipFree(out));
    CK(hipFree(meta));
    return 0;
}
