// Wire-format constants and the per-element codes (wire.hip's layout; include/flcodec.h), shared by
// the pack / decode kernels of wire.hip and the fused encode -> code kernel of codecs.hip.
#pragma once
#include "common.hpp"

namespace flc {

enum { FMT_F32 = 1, FMT_Q8 = 2, FMT_Q16 = 3, FMT_NAT16 = 4, FMT_SPARSE = 5, FMT_RANKK = 6 };
struct PayloadHeader {
    uint32_t fmt, count;
    float norm;
    uint32_t bad;          // elements whose code search failed (0 by construction)
};

__host__ __device__ inline int64_t a16(int64_t b) { return (b + 15) & ~int64_t(15); }

// ---- level codes ------------------------------------------------------------------------------
__device__ inline float lev_value(const float* lv, uint32_t idx, bool neg, float norm) {
    return copysignf(lv[idx], neg ? -1.f : 1.f) * norm;
}

__device__ inline uint32_t lev_code(float v, const float* lv, int s, float norm, uint32_t sbit, uint32_t* bad) {
    const uint32_t vb = __float_as_uint(v);
    if (vb == 0u) return 0u;                                   // +0 (x == 0)
    const bool neg = (vb >> 31) != 0u;
    if (v != v) return sbit;                                   // NaN: -0 * non-finite norm
    // the guess only has to land within one level: a product by 1 / norm, checked exactly below
    const float y = fabsf(v) * __builtin_amdgcn_rcpf(norm);
    int g = (int)rintf(y * (float)s);
    g = g < 0 ? 0 : (g > s ? s : g);
    for (int dlt = 0; dlt < 3; ++dlt) {
        const int c = dlt == 0 ? g : (dlt == 1 ? g - 1 : g + 1);
        if (c >= 0 && c <= s && __float_as_uint(lev_value(lv, (uint32_t)c, neg, norm)) == vb)
            return (neg ? sbit : 0u) | (uint32_t)c;
    }
    int lo = 0, hi = s;                                        // levels ascending: binary search on |v|
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        const float m = fabsf(lev_value(lv, (uint32_t)mid, neg, norm));
        if (__float_as_uint(lev_value(lv, (uint32_t)mid, neg, norm)) == vb) return (neg ? sbit : 0u) | (uint32_t)mid;
        if (m < fabsf(v)) lo = mid + 1; else hi = mid - 1;
    }
    atomicAdd(bad, 1u);
    return neg ? sbit : 0u;
}

// a level index past s (only a malformed message has one) reads the top level, never past the table
__device__ inline float lev_decode(uint32_t code, const float* lv, int s, float norm, uint32_t sbit) {
    if (code == 0u) return 0.f;
    return lev_value(lv, min(code & (sbit - 1u), (uint32_t)s), (code & sbit) != 0u, norm);
}

// ---- natural codes ----------------------------------------------------------------------------
__device__ inline uint32_t nat_code(float v) {
    const uint32_t vb = __float_as_uint(v), sg = (vb >> 31) << 15;
    if ((vb & 0x7FFFFFFFu) == 0u) return sg;
    if (v != v) return 0x7FFFu;
    if (isinf(v)) return sg | 0x7FFEu;
    int e;
    (void)frexpf(v, &e);                                       // |v| = 0.5 * 2^e (a power of two)
    return sg | (uint32_t)(e - 1 + 16384);
}

__device__ inline float nat_decode(uint32_t c) {
    const float sg = (c & 0x8000u) ? -1.f : 1.f;
    const uint32_t m = c & 0x7FFFu;
    if (m == 0u) return copysignf(0.f, sg);
    if (m == 0x7FFFu) return __uint_as_float(0x7FC00000u);
    if (m == 0x7FFEu) return copysignf(__builtin_inff(), sg);
    return copysignf(ldexpf(1.f, (int)m - 16384), sg);
}

}  // namespace flc
