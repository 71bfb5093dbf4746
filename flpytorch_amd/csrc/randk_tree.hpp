// Device-RNG RandK sampler: a uniformly random K-subset of [0, D) that is generated chunk by chunk.
//
// The reference draws S = rndgen.choice(D, K, replace=False) (compressors.py:206) — a uniform
// K-subset from numpy's stream; compat mode reproduces that stream bit for bit.  Device mode is this
// build's own keyed generator, built so that the chunk-owner fold can regenerate any chunk's members
// on the fly instead of bucketing K indices per row through memory:
//
//   1. per-chunk counts (chunk = 4096 elements): the multivariate hypergeometric law of a uniform
//      K-subset's chunk counts, drawn down a binary tree over the chunk range — node (l, i) covers
//      chunks [lo(l, i), lo(l, i + 1)) with lo(l, i) = floor(i C / 2^l); its m members split
//      m = x + (m - x) with x ~ Hypergeometric(population, left population, m), inverted from one
//      53-bit uniform keyed by (client key, node id 2^l + i);
//   2. inside chunk c, the first m_c images of a keyed 12-bit permutation (4-round Feistel on 6 + 6
//      bits, cycle-walked into a short last chunk): a uniform m_c-subset of the chunk.
// (Nodes with at most 64 members draw their split member by member with integer arithmetic.)
// Given exact hypergeometric counts and uniform within-chunk subsets, the union is a uniform K-subset
// (the law of choice(D, K, replace=False)); exactly K distinct indices, each kept with probability
// K / D (RandK's unbiasedness, compressors.py:136's w = D/K - 1).
//
// The hypergeometric probabilities are evaluated with Loader's saddle-point form (stirlerr / bd0 /
// dbinom_raw, the algorithm of R's dhyper), relative error ~1e-14, and the inversion walks from the
// mode with the exact pmf ratio recurrence.  Every operation is an IEEE +, -, *, / or an exact
// frexp / ldexp / floor, with log and exp written out here: the host mirror, the device kernels and
// the numpy restatement (oracle/devrng.py) produce the same bits (-ffp-contract=off).
#pragma once
#include <stdint.h>

#include <cmath>

#include "common.hpp"

namespace flc {
namespace rktree {

constexpr int CH_SHIFT = 12;                       // chunk = 4096 elements (CHUNK in chunks.hpp)
constexpr int64_t CH = (int64_t)1 << CH_SHIFT;

// ---- deterministic log / exp (double) ---------------------------------------------------------
constexpr double LN2_HI = 6.93147180369123816490e-01;   // 32 significant bits: k * LN2_HI exact
constexpr double LN2_LO = 1.90821492927058770002e-10;

__host__ __device__ inline double dlog(double x) {        // x > 0, finite
    int e;
    double m = frexp(x, &e);                               // x = m 2^e, m in [0.5, 1)
    if (m < 0.70710678118654752440) { m = m * 2.0; e = e - 1; }
    const double s = (m - 1.0) / (m + 1.0);                // |s| <= 0.1716
    const double z = s * s;
    double p = 1.0 / 25.0;                                  // log m = 2 atanh s = 2 (s + s^3/3 + ...)
    p = p * z + 1.0 / 23.0;
    p = p * z + 1.0 / 21.0;
    p = p * z + 1.0 / 19.0;
    p = p * z + 1.0 / 17.0;
    p = p * z + 1.0 / 15.0;
    p = p * z + 1.0 / 13.0;
    p = p * z + 1.0 / 11.0;
    p = p * z + 1.0 / 9.0;
    p = p * z + 1.0 / 7.0;
    p = p * z + 1.0 / 5.0;
    p = p * z + 1.0 / 3.0;
    const double lm = 2.0 * s + 2.0 * s * (z * p);
    const double de = (double)e;
    return de * LN2_HI + (lm + de * LN2_LO);
}

__host__ __device__ inline double dexp(double x) {
    if (!(x > -745.0)) return 0.0;                         // underflow (and NaN -> 0)
    const double kf = floor(x * 1.4426950408889634 + 0.5);
    const double r = (x - kf * LN2_HI) - kf * LN2_LO;      // |r| <= ~0.35
    double p = 1.0;                                         // Horner of the Taylor series to r^18 / 18!
    p = 1.0 + (r * p) * (1.0 / 18.0);
    p = 1.0 + (r * p) * (1.0 / 17.0);
    p = 1.0 + (r * p) * (1.0 / 16.0);
    p = 1.0 + (r * p) * (1.0 / 15.0);
    p = 1.0 + (r * p) * (1.0 / 14.0);
    p = 1.0 + (r * p) * (1.0 / 13.0);
    p = 1.0 + (r * p) * (1.0 / 12.0);
    p = 1.0 + (r * p) * (1.0 / 11.0);
    p = 1.0 + (r * p) * (1.0 / 10.0);
    p = 1.0 + (r * p) * (1.0 / 9.0);
    p = 1.0 + (r * p) * (1.0 / 8.0);
    p = 1.0 + (r * p) * (1.0 / 7.0);
    p = 1.0 + (r * p) * (1.0 / 6.0);
    p = 1.0 + (r * p) * (1.0 / 5.0);
    p = 1.0 + (r * p) * (1.0 / 4.0);
    p = 1.0 + (r * p) * (1.0 / 3.0);
    p = 1.0 + (r * p) * (1.0 / 2.0);
    p = 1.0 + r * p;
    return ldexp(p, (int)kf);
}

// ---- Loader's binomial / hypergeometric densities ---------------------------------------------
// stirlerr(n) = log(n!) - (n + 1/2) log n + n - log sqrt(2 pi), integer n >= 0 (0 -> 0)
__host__ __device__ inline double stirlerr(double n) {
    if (n <= 15.0) {                                        // a table read, no branch per value
        constexpr double T[16] = {0.0, 0.08106146679532726, 0.0413406959554093, 0.02767792568499834,
                                  0.020790672103765093, 0.016644691189821193, 0.013876128823070748,
                                  0.01189670994589177, 0.010411265261972096, 0.009255462182712733,
                                  0.00833056343336287, 0.007573675487951841, 0.00694284010720953,
                                  0.006408994188004207, 0.0059513701127588475, 0.005554733551962801};
        return T[(int)n];
    }
    const double S0 = 1.0 / 12.0, S1 = 1.0 / 360.0, S2 = 1.0 / 1260.0, S3 = 1.0 / 1680.0, S4 = 1.0 / 1188.0;
    const double nn = n * n;
    if (n > 500.0) return (S0 - S1 / nn) / n;
    if (n > 80.0) return (S0 - (S1 - S2 / nn) / nn) / n;
    if (n > 35.0) return (S0 - (S1 - (S2 - S3 / nn) / nn) / nn) / n;
    return (S0 - (S1 - (S2 - (S3 - S4 / nn) / nn) / nn) / nn) / n;
}

// The density code is called out of line (and its loops kept rolled): inlined into the tree walk it
// grew the counts kernel to ~15 K instructions, past the instruction cache.
#define RK_COLD __host__ __device__ inline __attribute__((noinline))

// deviance term x log(x / np) + np - x, by its series when x ~ np (|v| < 0.1: <= 17 terms)
RK_COLD double bd0(double x, double np) {
    if (fabs(x - np) < 0.1 * (x + np)) {
        double v = (x - np) / (x + np);
        double s = (x - np) * v;
        double ej = 2.0 * x * v;
        v = v * v;
        // 1 / (2j + 1), j = 1 ..
        constexpr double R[24] = {0.3333333333333333, 0.2, 0.14285714285714285, 0.1111111111111111,
                                  0.09090909090909091, 0.07692307692307693, 0.06666666666666667,
                                  0.058823529411764705, 0.05263157894736842, 0.047619047619047616,
                                  0.043478260869565216, 0.04, 0.037037037037037035, 0.034482758620689655,
                                  0.03225806451612903, 0.030303030303030304, 0.02857142857142857,
                                  0.02702702702702703, 0.02564102564102564, 0.024390243902439025,
                                  0.023255813953488372, 0.022222222222222223, 0.02127659574468085,
                                  0.02040816326530612};
#pragma unroll 1
        for (int j = 0; j < 24; ++j) {
            ej = ej * v;
            const double s1 = s + ej * R[j];
            if (s1 == s) return s1;
            s = s1;
        }
        return s;
    }
    return x * dlog(x / np) + np - x;
}

constexpr double LN_2PI = 1.8378770664093456;

RK_COLD double dbinom_raw(double x, double n, double p, double q) {
    if (p == 0.0) return x == 0.0 ? 1.0 : 0.0;
    if (q == 0.0) return x == n ? 1.0 : 0.0;
    if (x == 0.0) {
        if (n == 0.0) return 1.0;
        return dexp(p < 0.1 ? -bd0(n, n * q) - n * p : n * dlog(q));
    }
    if (x == n) return dexp(q < 0.1 ? -bd0(n, n * p) - n * q : n * dlog(p));
    if (x < 0.0 || x > n) return 0.0;
    const double lc = stirlerr(n) - stirlerr(x) - stirlerr(n - x) - bd0(x, n * p) - bd0(n - x, n * q);
    const double lf = LN_2PI + dlog(x) + dlog((n - x) / n);
    return dexp(lc - 0.5 * lf);
}

// P(X = x), X = successes among m draws without replacement from r successes and b failures:
// Loader's p1 p2 / p3 of three binomial densities (R's dhyper), with the three saddle-point terms
// combined under one exp and their three log factors under one log when x is interior
RK_COLD double dhyper(double x, double r, double b, double m) {
    if (x < 0.0 || m < x || r < x || m - x > b) return 0.0;
    if (m == 0.0) return x == 0.0 ? 1.0 : 0.0;
    const double N = r + b, p = m / N, q = (N - m) / N;
    const double y = m - x, z = b - y;                      // failures drawn / left
    if (x == 0.0 || x == r || y == 0.0 || z == 0.0 || m == N) {
        const double p1 = dbinom_raw(x, r, p, q);
        const double p2 = dbinom_raw(y, b, p, q);
        const double p3 = dbinom_raw(m, N, p, q);
        return p1 * p2 / p3;
    }
    const double lc = (stirlerr(r) - stirlerr(x) - stirlerr(r - x) - bd0(x, r * p) - bd0(r - x, r * q)) +
                      (stirlerr(b) - stirlerr(y) - stirlerr(z) - bd0(y, b * p) - bd0(z, b * q)) -
                      (stirlerr(N) - stirlerr(m) - stirlerr(N - m) - bd0(m, N * p) - bd0(N - m, N * q));
    const double lf = LN_2PI + dlog(((x * (r - x)) / r) * ((y * z) / b) * (N / (m * (N - m))));
    return dexp(lc - 0.5 * lf);
}

// Inversion of the hypergeometric law from u in [0, 1): the values are visited from the mode
// outwards (x0, x0 + 1, x0 - 1, x0 + 2, ...), u is reduced by each value's mass, and the value that
// takes u below 0 is returned — any fixed visiting order inverts the law exactly.
RK_COLD int64_t hyper_draw(int64_t N, int64_t r, int64_t m, double u) {
    if (m <= 0 || r <= 0) return 0;
    if (r >= N) return m;
    if (m >= N) return r;
    const int64_t xmin = m - (N - r) > 0 ? m - (N - r) : 0;
    const int64_t xmax = r < m ? r : m;
    if (xmin >= xmax) return xmin;
    int64_t x0 = (int64_t)floor(((double)m + 1.0) * ((double)r + 1.0) / ((double)N + 2.0));
    x0 = x0 < xmin ? xmin : (x0 > xmax ? xmax : x0);
    const double b = (double)(N - r), rr = (double)r, mm = (double)m, tail = (double)(N - r - m);
    const double p0 = dhyper((double)x0, rr, b, mm);
    u = u - p0;
    if (u < 0.0) return x0;
    int64_t lo = x0, hi = x0;
    double plo = p0, phi = p0;
    // Four steps per side at a time: their ratios are independent of the running masses, so the
    // divisions overlap; the masses are then updated and tested in the one-step order (the values
    // are those of the step-by-step walk).
    for (;;) {
        double ru[4], rd[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {   // P(x + 1) / P(x) = (r - x)(m - x) / ((x + 1)(N - r - m + x + 1))
            const double x = (double)(hi + k);
            ru[k] = ((rr - x) * (mm - x)) / ((x + 1.0) * (tail + x + 1.0));
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {   // P(x - 1) / P(x) = x (N - r - m + x) / ((r - x + 1)(m - x + 1))
            const double x = (double)(lo - k);
            rd[k] = (x * (tail + x)) / ((rr - x + 1.0) * (mm - x + 1.0));
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            bool moved = false;
            if (hi < xmax) {
                phi = phi * ru[k];
                ++hi;
                u = u - phi;
                if (u < 0.0) return hi;
                moved = true;
            }
            if (lo > xmin) {
                plo = plo * rd[k];
                --lo;
                u = u - plo;
                if (u < 0.0) return lo;
                moved = true;
            }
            // out of support, or both tails below 1e-18 (the rest of the mass is rounding residue)
            if (!moved || (phi < 1e-18 && plo < 1e-18)) return x0;
        }
    }
}

// ---- the tree over chunks ---------------------------------------------------------------------
__host__ __device__ inline int tree_depth(int64_t C) {     // smallest L with 2^L >= C
    int L = 0;
    while (((int64_t)1 << L) < C) ++L;
    return L;
}
__host__ __device__ inline int64_t node_lo(int64_t C, int l, int64_t i) { return (i * C) >> l; }
__host__ __device__ inline int64_t chunk_pop(int64_t a, int64_t b, int64_t d) {   // elements of chunks [a, b)
    const int64_t e = b * CH < d ? b * CH : d;
    return e - a * CH;
}
__host__ __device__ inline uint64_t tree_key(uint64_t ckey) { return mix64(ckey ^ 0x5851F42D4C957F2Dull); }

__host__ __device__ inline uint64_t mulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

// Few members (m <= SEQ_MAX): the m draws without replacement made one by one — draw s lands in the
// left part with probability remL / remT, decided by the 64-bit uniform u_s as
// floor(u_s remT / 2^64) < remL (exact up to 2^-64 per draw); integer arithmetic only.
constexpr int64_t SEQ_MAX = 64;
__host__ __device__ inline int64_t seq_draw(uint64_t nkey, int64_t N, int64_t r, int64_t m) {
    uint64_t remT = (uint64_t)N, remL = (uint64_t)r;
    int64_t x = 0;
    for (int64_t s = 0; s < m; ++s) {
        const uint64_t u = ((uint64_t)fmix32((uint32_t)nkey + 0x9E3779B1u * (uint32_t)(2 * s)) << 32) |
                           fmix32((uint32_t)(nkey >> 32) + 0x9E3779B1u * (uint32_t)(2 * s + 1));
        if (mulhi64(u, remT) < remL) { ++x; --remL; }
        --remT;
    }
    return x;
}

// split of node (l, i) holding m members: the left child's count
__host__ __device__ inline int64_t node_split(uint64_t tkey, int64_t C, int64_t d, int l, int64_t i, int64_t m) {
    if (m == 0) return 0;
    const int64_t a = node_lo(C, l, i), mid = node_lo(C, l + 1, 2 * i + 1), b = node_lo(C, l, i + 1);
    const int64_t pl = chunk_pop(a, mid, d), pr = chunk_pop(mid, b, d);
    if (pl == 0) return 0;
    if (pr == 0) return m;
    const int64_t node = ((int64_t)1 << l) + i;
    if (m <= SEQ_MAX) return seq_draw(mix64(tkey ^ (0x9E3779B97F4A7C15ull * (uint64_t)node)), pl + pr, pl, m);
    return hyper_draw(pl + pr, pl, m, uniform53(tkey, node));
}

// ---- the keyed permutation inside a chunk -----------------------------------------------------
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
        while (v >= len) v = once(v);                       // a short last chunk only
        return v;
    }
};

}  // namespace rktree
}  // namespace flc
