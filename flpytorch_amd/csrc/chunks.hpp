// Chunked-row helpers shared by the sparsifying paths (select.hip: TopK / RandK;
// dither_sparse.hip: sparse QSGD): chunk = 4096 elements = one wave's tile of 16 wave-loads.
#pragma once
#include "common.hpp"

namespace flc {

// Row counters of the candidate lists are reserved with atomics by every wave; counters of
// neighbouring rows sharing an L2 line serialise those atomics (measured: -10 % filter bandwidth,
// tools/probe_filter.hip), so each row's counter has a 128 B line of its own.
constexpr int RCS = 32;

// The folds' carried tiles (row groups after the first) loaded with all their loads in flight
// (k_chunk_accum, k_ds_accum); 0: the per-64-column load -> LDS write loop
#ifndef FLC_TILE_V4
#define FLC_TILE_V4 1
#endif

__host__ __device__ inline int64_t nchunks(int64_t d) { return (d + CHUNK - 1) >> CHUNK_SHIFT; }

// Buffer descriptor of one chunk built from the wave-uniform chunk base (SGPRs): 32-bit lane
// offsets, no 64-bit address VGPRs, and the hardware range check returns 0 past the row's end.
__device__ inline __amdgpu_buffer_rsrc_t chunk_rsrc(const float* r, int64_t j0, int64_t d) {
    const int64_t len = max((int64_t)0, min((int64_t)CHUNK, d - j0));
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(r + j0), (short)0, (int)(len * 4), 0x00020000);
}
// Cache policy of the streaming row loads (buffer aux bits; 2 = nt): every row element is read
// once per launch, so the lines are not worth keeping (measured on the C3 / C4 filters: 2-6 %
// faster than the default policy, box-dependent; an A/B build can set -DFLC_LOADPOL=0)
#ifndef FLC_LOADPOL
#define FLC_LOADPOL 2
#endif
__device__ inline float4 load_q(__amdgpu_buffer_rsrc_t rs, int lane, int L) {
    const auto q = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, L * 1024, FLC_LOADPOL);
    return make_float4(__uint_as_float(q[0]), __uint_as_float(q[1]), __uint_as_float(q[2]), __uint_as_float(q[3]));
}

// Range-checked descriptor of an entry list (cnt 32-bit words): loads past the end return 0.
__device__ inline __amdgpu_buffer_rsrc_t list_rsrc(const void* p, uint32_t cnt) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)(cnt * 4u), 0x00020000);
}

}  // namespace flc
