// Device-RNG RandK sampler: a uniformly random K-subset of [0, D), generated chunk by chunk.
//
// The reference draws S = rndgen.choice(D, K, replace=False) (compressors.py:206) — a uniform
// K-subset from numpy's stream; compat mode reproduces that stream bit for bit.  Device mode is this
// build's own keyed generator, built so that the chunk-owner fold can regenerate any chunk's members
// on the fly instead of bucketing K indices per row through memory:
//
//   1. per-chunk counts (chunk = 4096 elements): m_c = #{t < K : Pi(t) in chunk c} for a keyed
//      permutation Pi of [0, D) (balanced 4-round Feistel on 2h >= log2 D bits, cycle-walked into
//      [0, D)) — the chunk counts of the uniform K-subset Pi([0, K)), i.e. the multivariate
//      hypergeometric law; computed as a histogram, every t independent (no sequential chain);
//   2. inside chunk c, the first m_c images of a keyed 12-bit permutation (4-round Feistel on 6 + 6
//      bits, cycle-walked into a short last chunk): a uniform m_c-subset of the chunk.
// Counts with the law of a uniform K-subset plus uniform within-chunk subsets drawn with separate
// keys make the union a uniform K-subset (the law of choice(D, K, replace=False), in the
// ideal-permutation model the Feistel stands for): exactly K distinct indices, each kept with
// probability K / D (RandK's unbiasedness, compressors.py:136's w = D/K - 1).
//
// Integer arithmetic only: the host mirror (flc_device_randk_indices), the kernels and the numpy
// restatement (oracle/devrng.py) produce the same sets.
#pragma once
#include <stdint.h>

#include "common.hpp"

namespace flc {
namespace rktree {

constexpr int CH_SHIFT = 12;                       // chunk = 4096 elements (CHUNK in chunks.hpp)
constexpr int64_t CH = (int64_t)1 << CH_SHIFT;

// The row permutation Pi of [0, d): balanced Feistel on 2h bits (4^h >= d), round function
// fmix32(half ^ round key) masked to h bits, round keys from the client key.
struct RowPerm {
    uint32_t rkey[4];
    uint32_t half_bits, half_mask;
    uint64_t d;
    __host__ __device__ RowPerm(uint64_t ckey, uint64_t dd) : d(dd) {
        uint32_t b = 1;
        while ((1ull << (2 * b)) < dd) ++b;
        half_bits = b;
        half_mask = (b >= 32) ? 0xFFFFFFFFu : ((1u << b) - 1u);
        const uint64_t k = mix64(ckey ^ 0x5851F42D4C957F2Dull);
        for (int i = 0; i < 4; ++i) rkey[i] = (uint32_t)mix64(k + ((uint64_t)i << 56));
    }
    __host__ __device__ inline uint64_t once(uint64_t v) const {
        uint32_t l = (uint32_t)(v >> half_bits) & half_mask, r = (uint32_t)v & half_mask;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t nr = l ^ (fmix32(r ^ rkey[i]) & half_mask);
            l = r;
            r = nr;
        }
        return ((uint64_t)l << half_bits) | r;
    }
    __host__ __device__ inline uint64_t operator()(uint64_t t) const {
        uint64_t v = once(t);
        while (v >= d) v = once(v);                         // cycle walking stays inside [0, d)
        return v;
    }
};

// The keyed permutation inside chunk c (12 bits, 6 + 6), cycle-walked into a short last chunk
struct ChunkPerm {
    uint32_t k0, k1, k2, k3, len;
    __host__ __device__ ChunkPerm(uint64_t ckey, int64_t c, uint32_t n) : len(n) {
        const uint64_t b = mix64(ckey ^ (0xD1B54A32D192ED03ull * (uint64_t)(c + 1)));
        k0 = (uint32_t)b;
        k1 = (uint32_t)(b >> 32);
        k2 = fmix32(k0 ^ 0x3C6EF372u);
        k3 = fmix32(k1 + 0xA54FF53Au);
    }
    __host__ __device__ inline uint32_t once(uint32_t v) const {
        uint32_t l = v >> 6, r = v & 63u, t;
        t = l ^ (fmix32(r ^ k0) & 63u); l = r; r = t;
        t = l ^ (fmix32(r ^ k1) & 63u); l = r; r = t;
        t = l ^ (fmix32(r ^ k2) & 63u); l = r; r = t;
        t = l ^ (fmix32(r ^ k3) & 63u); l = r; r = t;
        return (l << 6) | r;
    }
    __host__ __device__ inline uint32_t operator()(uint32_t t) const {
        uint32_t v = once(t);
        while (v >= len) v = once(v);
        return v;
    }
};

}  // namespace rktree
}  // namespace flc
