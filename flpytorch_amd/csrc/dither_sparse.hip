// Sparse fused standard dithering / QSGD encode + reduce: device-RNG mode, p = 2 norm.
// fl_pytorch/utils/compressors.py:270-299 (the codec; qsgd = std dithering with p = 2, 95-101) and
// the serverGradient fold (algorithms.py:1748-1770), reading every client row from HBM ONCE.
//
// Why a sparse path: the encode needs the row's norm before any element, so the dense path reads
// every row twice (norm pass + encode pass, codecs.hip).  But QSGD's output is sparse: element j
// is nonzero only if y_j = |x_j| / ||x||_2 >= l1 (the first level, 1/s) or its draw goes up, so
//     E[nonzeros] <= sum_j min(1, y_j / l1) <= ||x||_1 / (l1 ||x||_2) <= s sqrt(D)
// for ANY row (2.0 % of the elements at s = 127, D = 25 M for Gaussian rows).  One streaming pass
// can therefore accumulate the norm AND decide almost every element, using BOUNDS n_lo <= n <=
// n_hi of the norm from a spread sample (checked once the norm is known; a row outside its bounds
// is folded dense):
//
//   sample  : per row, sum of squares (and 4th powers) of a spread 16 K-element sample -> n_lo,
//             n_hi, the candidate scale qc = 256 (1 + 2^-18) / (l1 n_lo), the classification
//             scales q0 = RU(1 / (l1 n_lo)), q1 = RD(1 / (l1 n_hi)), the device-RNG row key.
//   filter  : ONE pass over every row: float64 sum of squares per 8192-element item (fixed slots),
//             and every element passing  fma(|x|, qc, hi8) > 254.98  staged in LDS (hi8 = the top
//             byte of the element's draw, one group hash per 4 elements).  At the item's end each
//             staged candidate is classified with its full 32-bit draw h (the low hash computed
//             for the ~2 % staged only):
//               sure   — kept at level l1 for EVERY norm in [n_lo, n_hi]: a 2-byte entry
//                        (item-local index | sign) — its contribution is +-RN(l1 n) for any n;
//               drop   — zero for every norm >= n_lo: nothing written;
//               ambiguous (norm band, higher levels, 0-ish draws): the 8-byte (index | hi8, x).
//   final   : per row, norm = RN(sqrt(sum of the partials in a fixed order)); the row is folded
//             DENSE (every element re-read and encoded) if the norm is outside [n_lo, n_hi], not
//             finite, its weight not finite, or an item overflowed its staging.
//   resolve : the ambiguous entries encoded exactly with the norm (ds_encode = DitherOp::apply's
//             arithmetic), rewritten in place as (index, C(x)) when nonzero.
//   accum   : one wave owns a 2048-element half chunk as an fp32 LDS tile and folds the rows in
//             order: per row its sure entries (+-RN(l1 n)) and resolved entries (C(x)), times the
//             weight; untouched columns get the sign of zero the sequential fold of the all-zero
//             contributions gives (-0 only if every row gives -0).
//
// Exactness of the classification.  In the first level interval [0, l1] the encode keeps l1 iff
// h >= thr(n),  thr(n) = sat_u32(ceil(RN(RN(y - l1) / (-l1 2^-32)))),  y = RN(|x| / n).  Every
// step is monotone, so thr is nondecreasing in n; and |thr(n) - 2^32 (1 - |x| / (n l1))| <
// 2^32 2^-22.  Hence for n in [n_lo, n_hi] (and |x| q0 <= 1 - 2^-18, so y < l1 throughout):
//   h / 2^32 + |x| / (n_hi l1) >= 1 + 2^-22  =>  kept for every such n      (sure)
//   h / 2^32 + |x| / (n_lo l1) <  1 - 2^-22  =>  not kept for every such n  (drop)
// evaluated as fp32 fmas with q1 / q0 and floor / ceil of h / 2^32 at 2^-24 resolution against
// 1 +- 2^-20 (the fma's rounding is < 2^-24 there).  The candidate test itself is conservative (never
// drops a nonzero): for n >= n_lo a nonzero output has h >= p 2^32 with p >= 1 - y / l1 - 2^-23,
// so hi8 = h >> 24 > 255 - 256 |x| (1 + 2^-24) / (l1 n_lo) - 2^-15, and |x| qc + hi8 > 255 - 2^-15;
// the fp32 fma loses < 2^-14 there, so > 254.98 keeps every nonzero.  Elements in higher
// intervals (y >= l1) have |x| qc >= 256.
#include <map>
#include <mutex>
#include <type_traits>
#include <vector>

#include "chunks.hpp"
#include "codec_ops.hpp"

namespace flc {

constexpr uint32_t DS_DENSE = 1u, DS_FAST = 4u;
#ifndef FLC_DS_W2
#define FLC_DS_W2 1
#endif
constexpr int DS_FGS = 2;                  // chunks per filter work item (8192 elements)
constexpr int DS_NH = 2 * DS_FGS;          // fold tiles (half chunks) per item
constexpr int DS_GCAP = 512;               // staged candidates per item (6.25 %; more -> row overflow)
constexpr int DS_HCAP = DS_GCAP / DS_NH;    // entries per half chunk of an item (more -> row overflow)
constexpr int DS_MAXLEV = 15;              // entry level field: 4 bits (a higher level -> row dense)
#ifndef FLC_DS_SPLIT_SAMPLE
#define FLC_DS_SPLIT_SAMPLE 1         // QSGD row groups: only group 0's sample before the first filter
#endif
#ifndef FLC_DS_SMAX
#define FLC_DS_SMAX 65536
#endif
#ifndef FLC_DS_MARGIN
#define FLC_DS_MARGIN 0.02
#endif
constexpr int DS_SMAX = FLC_DS_SMAX;       // sample elements per row (256-element pieces)
constexpr int DS_SNT = 1024;               // sample threads per row
constexpr float DS_QT = 254.98f;
constexpr int DS_MAXS = 512;               // level table entries kept in LDS by the fold
constexpr uint32_t DS_OVF = 0xFFFFFFFFu;   // itm: the item overflowed its staging capacity
#ifndef FLC_DS_AP
#define FLC_DS_AP 16                // 16: measured 0.673 -> 0.622 ms at C4 (32: same as 16)
#endif
constexpr int DS_AP = FLC_DS_AP;           // rows of entry lists in flight in the fold
// rows per block of the filter's item order: 16 measured as fast as one block of all rows at C4
// (and 1, row-major, 1-2 % slower on the same box); a block never reads one row twice, so rows
// that alias (C5's replayed pool) are still read from HBM once per client
constexpr int64_t DS_RB = 16;
constexpr int DS_RINGC = 4;                // compat filter ring (x + u: 24 B per lane per step)
// Per-lane candidate staging (device-RNG filter): each lane appends its candidates to its own
// column of the wave's staging, slot row min(count, DS_PLS) (row DS_PLS absorbs a lane's
// overflow), so the per-element path has no cross-lane prefix (ballot / mbcnt) and no scalar
// counter chain; the columns are compacted once per item.  A lane with more than DS_PLS
// candidates in an item (Poisson(2.7) at C4: ~4e-3 of items) re-reads its elements afterwards.
#ifndef FLC_DS_PL
#define FLC_DS_PL 0
#endif
constexpr int DS_PLS = 10;
#ifndef FLC_DS_STPOL
// k_ds_filter's list copy-outs (sure and ambiguous entries) as nontemporal stores: bit-identical,
// C4 9.736 -> 9.615 ms per step on one allocation (profiles/r05/ab_list_stnt.txt; the same for
// the TopK filter's lists ran 7.618 -> 7.734 ms at C3, so FLC_TK_STPOL stays 0)
#define FLC_DS_STPOL 2
#endif
#ifndef FLC_DS_CU
#define FLC_DS_CU 2                  // k_ds_filter: candidate batches (of 64) classified per iteration
#endif
#ifndef FLC_DS_RW
#define FLC_DS_RW 8                  // k_ds_resolve: candidate windows (64 each) gathered up front
#endif

// One entry of the fold's lists (u16): half-chunk-local index (11 bits) | sign << 11 | level << 12;
// its contribution is copysign(levels[level], sign) * norm — C(x) exactly as the encode forms it.
struct DsWs {
    uint2* tabs;          // [Hp][N] (unused, count) of row's sure entries in half chunk h: the
                          // list of (h, row) is ent16[h][row][0 .. count + cntr)
    uint32_t* cntr;       // [Hp][N] resolved entries appended after them (k_ds_resolve)
    uint16_t* ent16;      // [Hp][N][DS_HCAP] entries, half-major: the fold of half h reads its
                          // rows' regions as one contiguous n * 256-byte run
    uint2* enta;          // [N][cap] ambiguous candidates (item-local index | hi8 << 13, x bits)
    uint32_t* itm;        // [G][N] ambiguous candidates of the item; DS_OVF: it overflowed
    uint32_t* flags;      // [N] DS_*
    float* qc;            // [N] candidate scale
    float* nlo;           // [N] norm bounds the classification assumes (checked by k_ds_final)
    float* nhi;
    float* q0;            // [N] RU(1 / (l1 n_lo))
    float* q1;            // [N] RD(1 / (l1 n_hi)); 0: no sure entries (n_hi unbounded)
    double* partial;      // [N][G] per-item sums of squares
    float* pn;            // [N] norm
    float* rpn;           // [N] RN(1 / norm)
    uint32_t* rk;         // [N] device-RNG row key
    float* part;          // [D] running sums carried between the row groups' folds
    float4* gtab;         // [DS_MAXS] level table (load_table) for the fold's dense rows, made by
                          // k_ds_sample: the fold keeps only its tile in LDS
    int64_t cap;          // per row: G * GCAP (each filter item owns a fixed region)
    int64_t G;            // filter items per row
    int64_t n;            // rows
};

constexpr int HCHUNK = CHUNK / 2;          // the fold's tile: 2048 elements (8 KB of LDS per wave)
__host__ __device__ inline int64_t nhalves(int64_t d) { return (d + HCHUNK - 1) / HCHUNK; }

// top byte of element j's draw (common.hpp dev_draw)
__device__ inline uint32_t ds_hi8(uint32_t j, uint32_t rk) { return (grouphash(j >> 2, rk) >> (8u * (j & 3u))) & 0xFFu; }
__device__ inline float f32_up(double v) { float f = (float)v; return (double)f < v ? nextafterf(f, __builtin_huge_valf()) : f; }
__device__ inline float f32_down(double v) { float f = (float)v; return (double)f > v ? nextafterf(f, 0.f) : f; }

// ------------------------------------------------------------------------------------------
// Sample: one workgroup per row.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(DS_SNT) void k_ds_sample(RowSrc rows, int64_t n, int64_t d, const float* __restrict__ levels,
                                                      int s, uint64_t seed, int64_t client0, DsWs ws, int64_t r_off) {
    constexpr int NW = DS_SNT / 64;
    __shared__ double r2[NW], r4[NW];
    const int64_t row = r_off + blockIdx.x;                               // (a launch may take a row range)
    if (row == 0) load_table(levels, s, ws.gtab);
    if (row >= n) return;
    const float* r = rows.row(row);
    double a2 = 0.0, a4 = 0.0;
    int64_t S;
    if (d <= DS_SMAX) {
        S = d;
        for (int64_t i = threadIdx.x; i < d; i += DS_SNT) {
            const double v = (double)r[i] * (double)r[i];
            a2 += v;
            a4 += v * v;
        }
    } else {
        // P pieces of 256 contiguous elements spread evenly; the block's 4 quarters take every 4th
        // piece, thread t reading element t % 256 of 16 pieces per round trip
        constexpr int P = DS_SMAX / 256, Q = DS_SNT / 256, U = 16;
        static_assert(P % (Q * U) == 0, "sample pieces");
        S = DS_SMAX;
        const int e = threadIdx.x & 255, q = threadIdx.x >> 8;
        for (int p0 = q; p0 < P; p0 += Q * U) {
            float x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) x[u] = r[((int64_t)(p0 + Q * u) * (d - 256)) / (P - 1) + e];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const double v = (double)x[u] * (double)x[u];
                a2 += v;
                a4 += v * v;
            }
        }
    }
    a2 = wave_sum(a2);
    a4 = wave_sum(a4);
    if ((threadIdx.x & 63) == 0) { r2[threadIdx.x >> 6] = a2; r4[threadIdx.x >> 6] = a4; }
    __syncthreads();
    if (threadIdx.x == 0) {
        a2 = 0.0;
        a4 = 0.0;
        for (int w = 0; w < NW; ++w) { a2 += r2[w]; a4 += r4[w]; }
        const float l0 = levels[0], l1 = levels[1];
        const bool bad = !(l0 == 0.f) || !(l1 > 0.f);   // the bounds need levels 0 < l1 < ...
        double nlo, nhi = __builtin_huge_val();
        if (S == d) {
            nlo = sqrt(a2) * (1.0 - 0x1p-20);              // the whole row: the norm itself
            nhi = sqrt(a2) * (1.0 + 0x1p-20);
        } else {
            // estimate of the sum of squares, discounted by 6 sigma of the sample mean + a margin; the
            // upper bound only for light-tailed samples (heavy tails: n_hi unbounded, no sure entries)
            const double m = (double)S, mean2 = a2 / m;
            const double var = fmax(a4 / m - mean2 * mean2, 0.0);
            const double rel = sqrt(var / m) / mean2;      // NaN/inf when mean2 == 0 or overflow
            const double f = fmin(fmax(1.0 - 6.0 * rel - FLC_DS_MARGIN, 0.25), 0.97);
            nlo = sqrt(f * mean2 * (double)d);
            if (rel <= 0.05) nhi = sqrt((1.0 + 6.0 * rel + FLC_DS_MARGIN) * mean2 * (double)d);
        }
        float nlof = (float)nlo;
        if (!(nlof >= 0.f) || !(nlof <= 3.0e38f)) nlof = 0.f;
        float nhif = f32_up(nhi);
        if (!(nhif >= nlof) || !(nhif <= 3.0e38f)) nhif = __builtin_huge_valf();
        const double qcd = 256.0 * (1.0 + 0x1p-18) / ((double)l1 * (double)nlof);   // +inf for nlof 0
        float qc = (float)(qcd * (1.0 + 0x1p-22));         // rounded up past the conversion
        if (!(qc >= 0.f)) qc = __builtin_huge_valf();
        float q0 = f32_up(1.0 / ((double)l1 * (double)nlof));                       // +inf for nlof 0
        float q1 = f32_down(1.0 / ((double)l1 * (double)nhif));                     // 0 for nhi inf
        if (!(q0 >= 0.f)) q0 = __builtin_huge_valf();
        if (!(q1 >= 0.f) || !(q1 <= 3.0e38f)) q1 = 0.f;
        if (bad) { qc = 0.f; q1 = 0.f; }                   // row is folded dense anyway
        ws.qc[row] = qc;
        ws.nlo[row] = nlof;
        ws.nhi[row] = nhif;
        ws.q0[row] = q0;
        ws.q1[row] = q1;
        ws.flags[row] = bad ? DS_DENSE : 0u;
        ws.rk[row] = rowkey(client_key(seed, client0 + row));
    }
}

// ------------------------------------------------------------------------------------------
// Filter: a RING-deep buffer-load pipeline across chunks and items (select.hip's TopK filter
// structure), the dithering candidate test and the norm.  A work item is DS_FGS consecutive
// 4096-element chunks of one row; its candidates are compacted (ballot / mbcnt) into wave-private
// LDS, classified (sure / drop / ambiguous) and copied out coalesced into the item's FIXED regions
// of the row's lists (item * GCAP): no reservation atomic, so nothing returning sits in the
// in-order vmcnt queue of the load stream.  The tab gets the sure entries' (offset, count) per
// 2048-element half chunk (the fold's tile).
// ------------------------------------------------------------------------------------------
// PROBE (tuning / A/B builds only, FLC_DS_PROBE or -DFLC_DS_PROBE_DEF; outputs NOT valid): 1 fp32
// norm; 2 no candidate staging; 3 loads + norm only; 4 the draw's group hash without its
// multiplies; 5 exec-narrowed staging without a branch; 6 staging without the classification
//
// COMPAT: the draws are the caller's float64 uniforms u (the reference's numpy stream, [n][uld]),
// read in the same single pass (12 B per element).  A lane then holds elements {2l, 2l+1, 128 + 2l,
// 128 + 2l + 1} of each 256-element step (one 512-B x load and one 1-KB u load per pair, both
// contiguous); the candidate test takes RN(u) * 256 for the top byte, and each staged candidate
// carries RD(u) (LDS) for its classification — the same bounds with h / 2^32 replaced by u, whose
// float brackets [RD(u), next float up] are tighter than the 24-bit h's.
struct CSlot {
    float2 xa, xb;       // elements 2l, 2l+1 | 128 + 2l, 128 + 2l + 1 of the step
    double2 ua, ub;      // their uniforms
};
__device__ inline CSlot load_c(__amdgpu_buffer_rsrc_t rx, __amdgpu_buffer_rsrc_t ru, int lane, int L) {
    CSlot s;
    const auto a = __builtin_amdgcn_raw_buffer_load_b64(rx, lane * 8, L * 1024, FLC_LOADPOL);
    const auto b = __builtin_amdgcn_raw_buffer_load_b64(rx, lane * 8 + 512, L * 1024, FLC_LOADPOL);
    const auto p = __builtin_amdgcn_raw_buffer_load_b128(ru, lane * 16, L * 2048, FLC_LOADPOL);
    const auto q = __builtin_amdgcn_raw_buffer_load_b128(ru, lane * 16 + 1024, L * 2048, FLC_LOADPOL);
    s.xa = make_float2(__uint_as_float(a[0]), __uint_as_float(a[1]));
    s.xb = make_float2(__uint_as_float(b[0]), __uint_as_float(b[1]));
    s.ua = make_double2(__hiloint2double((int)p[1], (int)p[0]), __hiloint2double((int)p[3], (int)p[2]));
    s.ub = make_double2(__hiloint2double((int)q[1], (int)q[0]), __hiloint2double((int)q[3], (int)q[2]));
    return s;
}
// descriptor of chunk c's uniforms (range-checked like chunk_rsrc: 0 past the row end)
__device__ inline __amdgpu_buffer_rsrc_t chunk_ursrc(const double* u, int64_t j0, int64_t d) {
    const int64_t len = max((int64_t)0, min((int64_t)CHUNK, d - j0));
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(u + j0), (short)0, (int)(len * 8), 0x00020000);
}
#ifndef FLC_DS_WPE
#define FLC_DS_WPE 6                 // 6 waves per SIMD (80 VGPRs): measured 9.19 -> 9.10 ms at C4 vs 5
#endif
#ifndef FLC_DS_WPEC
#define FLC_DS_WPEC 5                // compat: 5 (LDS: 32 KB of staging per block)
#endif
template <int RING, int GCAP, int PROBE = 0, bool COMPAT = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(COMPAT ? FLC_DS_WPEC : FLC_DS_WPE))) void k_ds_filter(RowSrc rows, int64_t n, int64_t r0, int64_t rn, int64_t rb, int64_t d, DsWs ws, UniformSrc us) {
    constexpr int FGS = DS_FGS, NH = DS_NH;
    static_assert(16 % RING == 0, "ring must divide the 16 loads of a chunk");
    static_assert(GCAP % 512 == 0 && (GCAP & (GCAP - 1)) == 0, "copy-out in whole 16-B wave slots; wrap mask");
    static_assert(!COMPAT || PROBE == 0, "probes: device-RNG filter only");
    constexpr int DS_ITEM_STORES = 4 + GCAP / 128;   // partial, itm, tab, sure and ambiguous copy-outs
    // (entry word, x bits); 64 slots past GCAP take the writes of a wave-instruction that starts
    // at GCAP (its item has overflowed)
    // per-lane staging (PL): DS_PLS + 1 slot rows of 64 lanes, compacted in place into the item's
    // list; its sure entries (4 halves x DS_HCAP u16 = 1 KB) then go to entries [GCAP, GCAP + 128)
    constexpr bool PL = FLC_DS_PL && !COMPAT && PROBE == 0;
    constexpr int SROWS = PL ? (DS_PLS + 1) * 64 : GCAP + 64;
    static_assert(!PL || (SROWS >= GCAP + 128 && DS_PLS * 64 >= GCAP / 2), "per-lane staging layout");
    __shared__ __attribute__((aligned(16))) uint2 stage[4][SROWS];
    __shared__ __attribute__((aligned(16))) uint16_t stage16[4][PL ? 8 : GCAP];
    __shared__ float stagef[4][COMPAT ? GCAP + 64 : 1];     // compat: RD(u) of the staged
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t G = ws.G;
    const int64_t items = rn * G;                            // this launch's rows: [r0, r0 + rn)
    const int64_t stride = (int64_t)gridDim.x * 4;
    int64_t it = (int64_t)blockIdx.x * 4 + wv;
    if (it >= items) return;
    const uint32_t lphi = (uint32_t)lane * 0x9E3779B1u;    // group index g = c*1024 + 64 L + lane
    uint2* sg = stage[wv];
    uint16_t* s16 = PL ? reinterpret_cast<uint16_t*>(stage[wv] + GCAP) : stage16[wv];
    float* sgf = stagef[wv];
    // LDS byte address of the wave's staging buffer (wave-uniform)
    const uint32_t sla = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(__attribute__((address_space(3))) uint2*)sg);
    typedef typename std::conditional<COMPAT, CSlot, float4>::type Slot;
    Slot ring[RING];
    // item order: blocks of rb rows (the last one shorter), and inside a block (gi, row) with the
    // row fastest: the waves in flight at any time read the same item of the block's rows, spread
    // over rb rows rather than one row's neighbouring items, and each row is read once per launch
    // even when rows alias (a row read twice inside one block would be served from the caches)
    auto item_at = [&](int64_t t, int64_t& r, int64_t& g) {
        const int64_t blk = t / (rb * G), rem = t - blk * rb * G;
        const int64_t bn = min(rb, rn - blk * rb);            // rows in this block
        g = rem / bn;
        r = r0 + blk * rb + (rem - g * bn);
    };
    int64_t row, gi0;
    item_at(it, row, gi0);
    int64_t c = gi0 * FGS;
    auto rs = chunk_rsrc(rows.row_s(row), c * CHUNK, d);
    auto urow = [&](int64_t r) { return us.u + r * us.uld; };
    auto ru = rs;
    if constexpr (COMPAT) ru = chunk_ursrc(urow(row), c * CHUNK, d);
#pragma unroll
    for (int L = 0; L < RING - 1; ++L) {
        if constexpr (COMPAT) ring[L] = load_c(rs, ru, lane, L);
        else ring[L] = load_q(rs, lane, L);
        __builtin_amdgcn_sched_barrier(0);
    }
    {
        // the stores an item ends with, dropped (num_records 0): the loop is entered with the same
        // vmcnt queue shape as it is re-entered
        const auto nd = __builtin_amdgcn_make_buffer_rsrc(ws.enta, (short)0, 0, 0x00020000);
#pragma unroll
        for (int k = 0; k < DS_ITEM_STORES; ++k) __builtin_amdgcn_raw_buffer_store_b32(0u, nd, lane * 4, k * 256, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
    while (it < items) {
        const float qc = sload(ws.qc + row);
        const uint32_t rk = sload(ws.rk + row);
        const int64_t gi = c / FGS;
        const int64_t nit = it + stride;
        uint32_t cnt = 0;
        uint32_t lcnt = 0;                                   // PL: this lane's candidates in the item
        double a2 = 0.0;
        int64_t nrow = row, nc = c;
#pragma unroll
        for (int sub = 0; sub < FGS; ++sub, ++c) {
            const int64_t j0 = c * CHUNK;
            __amdgpu_buffer_rsrc_t rsn, run = ru;
            if (sub + 1 < FGS) {
                rsn = chunk_rsrc(rows.row_s(row), j0 + CHUNK, d);
                if constexpr (COMPAT) run = chunk_ursrc(urow(row), j0 + CHUNK, d);
            } else if (nit < items) {
                int64_t ngi;
                item_at(nit, nrow, ngi);
                nc = ngi * FGS;
                rsn = chunk_rsrc(rows.row_s(nrow), nc * CHUNK, d);
                if constexpr (COMPAT) run = chunk_ursrc(urow(nrow), nc * CHUNK, d);
            } else {
                    rsn = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(rows.row_s(row)), (short)0, 0, 0x00020000);
                    if constexpr (COMPAT) run = chunk_ursrc(urow(row), 0, 0);
                }
                if constexpr (COMPAT) {
                    // item-local index of (L, q): 4096 sub + 2 lane + 256 L + {0, 1, 128, 129}[q]
                    uint32_t jb = (uint32_t)lane * 2u + (uint32_t)sub * CHUNK;
                    asm volatile("" : "+v"(jb));
#pragma unroll
                    for (int L = 0; L < 16; ++L) {
                        const int P = L + RING - 1;
                        ring[P % RING] = P < 16 ? load_c(rs, ru, lane, P) : load_c(rsn, run, lane, P - 16);
                        const CSlot sl = ring[L % RING];
                        const float vq[4] = {sl.xa.x, sl.xa.y, sl.xb.x, sl.xb.y};
                        const double uq[4] = {sl.ua.x, sl.ua.y, sl.ub.x, sl.ub.y};
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            a2 = fma((double)vq[q], (double)vq[q], a2);
                            const float hf = (float)uq[q];                 // RN(u): |hf - u| <= 2^-25
                            const bool f = fmaf(fabsf(vq[q]), qc, hf * 256.f) > DS_QT;
                            const uint64_t m = __ballot(f);
                            if (f) {
                                const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                                const uint32_t slot = min(cnt, (uint32_t)GCAP) + pre;
                                sg[slot] = make_uint2(jb + (uint32_t)(L * 256 + (q & 1) + (q >> 1) * 128), __float_as_uint(vq[q]));
                                // RD(u) (u in [0, 1): hf > u implies hf > 0)
                                sgf[slot] = (double)hf > uq[q] ? __uint_as_float(__float_as_uint(hf) - 1u) : hf;
                            }
                            cnt += (uint32_t)__popcll(m);
                        }
                        asm volatile("" : "+v"(a2));
                    }
                } else {
                // item-local index of (L, q): 4096 sub + 4 lane + 256 L + q (opaque: keeps the 64
                // constants out of VGPRs); the draw's top byte is recomputed for the staged only
                uint32_t jb = (uint32_t)lane * 4u + (uint32_t)sub * CHUNK;
                asm volatile("" : "+v"(jb));
                const uint32_t gb = lphi + (uint32_t)(c * 1024) * 0x9E3779B1u + rk;   // hash input of L = 0
#pragma unroll
                for (int L = 0; L < 16; ++L) {
                    const int P = L + RING - 1;
                    ring[P % RING] = P < 16 ? load_q(rs, lane, P) : load_q(rsn, lane, P - 16);
                    const float4 x = ring[L % RING];
                    uint32_t hg;
                    if (PROBE == 4) { hg = gb + (uint32_t)(L * 64) * 0x9E3779B1u; hg ^= hg >> 15; }   // cost probe only
                    else hg = gmix(gb + (uint32_t)(L * 64) * 0x9E3779B1u);
                    const float vq[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        if (PROBE == 1) a2 = (double)fmaf(vq[q], vq[q], (float)a2);
                        else a2 = fma((double)vq[q], (double)vq[q], a2);
                        if (PROBE == 3) continue;
                        const float hi = (float)((hg >> (8 * q)) & 0xFFu);
                        // no range test: past the row end the loads return 0, and a zero candidate
                        // is dropped; NaN from 0 * inf (qc = inf) is not a candidate
                        const bool f = fmaf(fabsf(vq[q]), qc, hi) > DS_QT;
                        const uint64_t m = PL ? 0ull : __ballot(f);
                        // exec-masked store (a branch-free store of every element to a per-lane spill
                        // slot measured 9.2 -> 11.9 ms: the staging is LDS-issue sensitive)
                        if (PROBE == 5) {
                            // A/B: the staging store without a branch — exec narrowed to the
                            // candidates for the one ds_write2 (the loop runs with every lane active)
                            const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                            uint32_t sb = sla + min(cnt, (uint32_t)GCAP) * 8u;
                            asm volatile("" : "+s"(sb));
                            const uint32_t la = sb + pre * 8u;
                            uint64_t saved;
                            asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, %1\n\ts_nop 1\n\t"
                                         "ds_write2_b32 %2, %3, %4 offset1:1\n\ts_mov_b64 exec, %0"
                                         : "=&s"(saved) : "s"(m), "v"(la), "v"(jb + (uint32_t)(L * 256 + q)), "v"(__float_as_uint(vq[q]))
                                         : "memory");
                        } else if (PL) {
                            // the lane's own column: slot row min(lcnt, DS_PLS), 512 B per row
                            const uint32_t la = sla + (uint32_t)lane * 8u + min(lcnt, (uint32_t)DS_PLS) * 512u;
                            if (f)
                                asm volatile("ds_write2_b32 %0, %1, %2 offset1:1" ::"v"(la), "v"(jb + (uint32_t)(L * 256 + q)),
                                             "v"(__float_as_uint(vq[q])) : "memory");
                            lcnt += f ? 1u : 0u;
                            continue;
                        } else if (PROBE != 2 && f) {
#if FLC_DS_W2
                            // slot = min(cnt, GCAP) + candidates in lower lanes (< GCAP + 64): exact
                            // while the item fits; past GCAP the item overflows (its row is folded
                            // dense) and the writes land in the spare slots.  The scalar part is folded
                            // into the wave's LDS address in SALU (sla), the lane part is one mbcnt
                            // pair; index and x go out as one ds_write2_b32 (no register pair to
                            // assemble for a 64-bit store).
                            const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                            uint32_t sb = sla + min(cnt, (uint32_t)GCAP) * 8u;
                            asm volatile("" : "+s"(sb));             // stays a scalar term: one v_lshl_add
                            const uint32_t la = sb + pre * 8u;
                            asm volatile("ds_write2_b32 %0, %1, %2 offset1:1" ::"v"(la), "v"(jb + (uint32_t)(L * 256 + q)),
                                         "v"(__float_as_uint(vq[q])) : "memory");
#else
                            const uint32_t pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, cnt)) & (GCAP - 1);
                            sg[pos] = make_uint2(jb + (uint32_t)(L * 256 + q), __float_as_uint(vq[q]));
#endif
                        }
                        cnt += (uint32_t)__popcll(m);
                    }
                    // keep the norm's fma chain here: left alone, the compiler sinks all 128 of an
                    // item's fmas to its end and holds the 128 x values live (218 VGPRs)
                    asm volatile("" : "+v"(a2));
                }
            }
            rs = rsn;
            ru = run;
        }
        a2 = wave_sum(a2);                                   // fixed butterfly: deterministic
        if constexpr (PL) {
            // Compaction in place: slot row k of every lane with more than k candidates, in row
            // order, lanes in order within a row.  An entry's new position never exceeds its slot
            // (k * 64 + lane) and a row is read before any of it is written, so nothing unread is
            // overwritten.  (The list order is free: k_ds_resolve / k_ds_accum do not depend on it.)
            const uint32_t lc = min(lcnt, (uint32_t)DS_PLS);
            for (uint32_t k = 0; k < (uint32_t)DS_PLS; ++k) {
                const bool v = k < lc;
                const uint64_t mk = __ballot(v);
                if (mk == 0) break;
                if (v) {
                    const uint32_t pos = cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u));
                    const uint2 e = sg[k * 64 + lane];
                    sg[pos] = e;
                }
                cnt += (uint32_t)__popcll(mk);
            }
            // Lanes past DS_PLS (rare): their candidates from #DS_PLS on were absorbed by the last
            // row; re-read those lanes' elements of the item and append them (the loads wait
            // behind the ring's, once)
            const bool ovl = lcnt > (uint32_t)DS_PLS;
            if (__ballot(ovl)) {
                if (cnt + 0u <= (uint32_t)GCAP) {
                    // one element per step, nothing unrolled: the ring (the next item's loads in
                    // flight) stays live in registers across this path
                    const int64_t cg = gi * FGS;
                    uint32_t seen = 0;
#pragma unroll 1
                    for (int e = 0; e < FGS * 64; ++e) {
                        const int sub = e >> 6, L = (e >> 2) & 15, q = e & 3;
                        const auto rso = chunk_rsrc(rows.row_s(row), (cg + sub) * CHUNK, d);
                        const float x = ovl ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rso, lane * 16 + q * 4, L * 1024, 0)) : 0.f;
                        const uint32_t hg = gmix(lphi + (uint32_t)((cg + sub) * 1024 + L * 64) * 0x9E3779B1u + rk);
                        const float hi = (float)((hg >> (8 * q)) & 0xFFu);
                        const bool f = ovl && fmaf(fabsf(x), qc, hi) > DS_QT;
                        const bool extra = f && seen >= (uint32_t)DS_PLS;
                        seen += f ? 1u : 0u;
                        const uint64_t me = __ballot(extra);
                        const uint32_t pos = cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(me >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)me, 0u));
                        if (extra && pos < (uint32_t)GCAP + 64u)
                            sg[pos] = make_uint2((uint32_t)(sub * CHUNK + L * 256 + q) + (uint32_t)lane * 4u, __float_as_uint(x));
                        cnt += (uint32_t)__popcll(me);
                    }
                } else {
                    cnt = GCAP + 1;                          // the item overflows anyway
                }
            }
        }
        const bool fits = cnt <= GCAP;
        const uint32_t base = (uint32_t)gi * GCAP;
        // Classification of the staged candidates (LDS and ALU only: no vector-memory op between
        // the item's loads and its fixed store sequence).  Sure entries go to stage16, half h's at
        // h * DS_HCAP; ambiguous ones are compacted in place in sg (a batch reads its 64 slots
        // before it writes lower ones).
        uint32_t na = 0;
        uint32_t hs[NH];
#pragma unroll
        for (int u = 0; u < NH; ++u) hs[u] = 0;
        {
            const float q0 = sload(ws.q0 + row), q1 = sload(ws.q1 + row);
            const uint32_t rk2 = rk ^ 0x27D4EB2Fu;
            const uint32_t j0 = (uint32_t)(gi * (FGS * CHUNK));
            const uint32_t ncl = (fits && PROBE != 6) ? cnt : 0u;     // probe 6: no classification
            // CU batches of 64 per iteration: their LDS reads and draw hashes are independent, so
            // they overlap; only the compaction (ballot / mbcnt counters) runs batch after batch.
            // All CU batches are read before any in-place write (writes go below e0 + 64 CU).
            constexpr int CU = FLC_DS_CU;
            for (uint32_t e0 = 0; e0 < ncl; e0 += 64 * CU) {
                uint2 en[CU];
                float hf[CU], hfu[CU];
                uint32_t hi8[CU];
                bool vv[CU];
#pragma unroll
                for (int b = 0; b < CU; ++b) {
                    const uint32_t e = e0 + (uint32_t)(b * 64 + lane);
                    vv[b] = e < ncl;
                    en[b] = vv[b] ? sg[e] : make_uint2(0u, 0u);
                }
#pragma unroll
                for (int b = 0; b < CU; ++b) {
                    const uint32_t loc = en[b].x & 0x1FFFu;
                    hi8[b] = 0;
                    if constexpr (COMPAT) {
                        const uint32_t e = e0 + (uint32_t)(b * 64 + lane);
                        const float ud = vv[b] ? sgf[e] : 0.f;
                        hf[b] = ud;
                        hfu[b] = __uint_as_float(__float_as_uint(ud) + 1u);
                    } else {
                        hi8[b] = ds_hi8(j0 + loc, rk);
                        const uint32_t h24 = (hi8[b] << 16) | (fmix32(colbase(j0 + loc) + rk2) >> 16);   // h >> 8
                        hf[b] = (float)h24 * 0x1p-24f;                      // hf <= draw / 2^32 <= hfu
                        hfu[b] = (float)(h24 + 1u) * 0x1p-24f;
                    }
                }
#pragma unroll
                for (int b = 0; b < CU; ++b) {
                    if (e0 + (uint32_t)(b * 64) >= ncl) break;       // wave-uniform
                    const float x = __uint_as_float(en[b].y), ax = fabsf(x);
                    const uint32_t loc = en[b].x & 0x1FFFu;
                    const bool inl = ax * q0 <= 1.0f - 0x1p-18f;
                    const bool nz = vv[b] && !(x == 0.f);
                    const bool sure = nz && inl && fmaf(ax, q1, hf[b]) >= 1.0f + 0x1p-20f;
                    const bool drop = !nz || (inl && fmaf(ax, q0, hfu[b]) < 1.0f - 0x1p-20f);
                    const bool amb = !sure && !drop;
                    const uint32_t u = loc >> 11;
                    uint32_t pin = 0;
#pragma unroll
                    for (int h = 0; h < NH; ++h) {
                        const uint64_t mh = __ballot(sure && u == (uint32_t)h);
                        const uint32_t ph = __builtin_amdgcn_mbcnt_hi((uint32_t)(mh >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mh, hs[h]));
                        pin = u == (uint32_t)h ? ph : pin;
                        hs[h] += (uint32_t)__popcll(mh);
                    }
                    if (sure && pin < (uint32_t)DS_HCAP)
                        s16[u * DS_HCAP + pin] = (uint16_t)((loc & (HCHUNK - 1)) | ((en[b].y >> 31) << 11) | (1u << 12));
                    const uint64_t ma = __ballot(amb);
                    const uint32_t pa = __builtin_amdgcn_mbcnt_hi((uint32_t)(ma >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ma, na));
                    if (amb) sg[pa] = make_uint2(loc | (hi8[b] << 13), en[b].y);      // k_ds_resolve's entry
                    na += (uint32_t)__popcll(ma);
                }
            }
        }
        bool ovf = !fits;
#pragma unroll
        for (int u = 0; u < NH; ++u) ovf |= hs[u] > (uint32_t)DS_HCAP;
        // The item's stores: a FIXED sequence of DS_ITEM_STORES vector-memory ops with no exec
        // branch (every lane stores; duplicate lanes write equal values to equal addresses; the
        // copy-outs are range-checked by their buffer descriptors).  The stores sit in the
        // in-order vmcnt queue in front of the loads issued after them; with one fixed sequence on
        // every path (the prologue issues the same count of dropped stores) the compiler's static
        // vmcnt waits count them exactly instead of draining part of the ring.
        ws.partial[row * G + gi] = a2;
        ws.itm[gi * n + row] = ovf ? DS_OVF : na;
        {
            const uint32_t u = (uint32_t)lane & (NH - 1);
            uint32_t hc = 0;
#pragma unroll
            for (int v = 0; v < NH; ++v) hc = (uint32_t)v == u ? hs[v] : hc;
            // halves past the row end land in the tab's padding rows (G * NH >= H)
            ws.tabs[(gi * NH + u) * n + row] = make_uint2(0u, ovf ? 0u : hc);
        }
        {
            // sure entries: lane l holds entries 8 (l % 16) .. + 8 of half l / 16; slots past the
            // half's count are sent out of range (dropped) by their offset, not by an exec branch
            static_assert(DS_HCAP == 128 && GCAP == 512, "sure copy-out: 16 lanes x 16 B per half");
            const uint32_t u = (uint32_t)lane >> 4, k8 = ((uint32_t)lane & 15u) * 8u;
            uint32_t hc = 0;
#pragma unroll
            for (int v = 0; v < NH; ++v) hc = (uint32_t)v == u ? hs[v] : hc;
            const bool put = !ovf && k8 < hc;
            // half u's region of this row: ent16[gi * NH + u][row], n * DS_HCAP entries apart
            const uint32_t hstride = (uint32_t)n * (DS_HCAP * 2);               // bytes
            const auto od = __builtin_amdgcn_make_buffer_rsrc(ws.ent16 + ((int64_t)gi * NH * n + row) * DS_HCAP, (short)0,
                                                              (int)((NH - 1) * hstride + DS_HCAP * 2), 0x00020000);
            const uint4 v = reinterpret_cast<const uint4*>(s16)[lane];
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v), od,
                                                   put ? u * hstride + k8 * 2u : 0x7FFFFFF0u, 0, FLC_DS_STPOL);
        }
        {
            // ambiguous entries: two per lane per 16-B store; an odd count's last slot is stale
            const uint32_t nrec = ovf ? 0u : ((na + 1u) & ~1u) * 8u;
            const auto od = __builtin_amdgcn_make_buffer_rsrc(ws.enta + row * ws.cap + base, (short)0, (int)nrec, 0x00020000);
            const uint4* sq = reinterpret_cast<const uint4*>(sg);
#pragma unroll
            for (int k = 0; k < GCAP / 128; ++k) {
                const uint4 v = sq[k * 64 + lane];
                __builtin_amdgcn_raw_buffer_store_b128(
                    __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v), od, (k * 64 + lane) * 16, 0, FLC_DS_STPOL);
            }
        }
        // the copy-out reads precede the next item's staging writes in the wave's program order
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        it = nit;
        row = nrow;
        c = nc;
    }
}

// ------------------------------------------------------------------------------------------
// Filter v2 (device draws, the product path): the same single pass, with each item's
// classification moved into the NEXT item's streaming loop.  Probes on one allocation (round 4):
// the classification epilogue cost k_ds_filter 1.25 ms of 9.69 at C4 (without it 8.44; loads +
// norm alone 8.36) — while a wave classifies it issues no loads, and the issue-bound epilogue
// grows on boxes that run a lower sustained clock.  Here the staging is double-buffered: item i
// is staged into buffer `par` while item i-1's candidates (buffer par ^ 1) are classified one
// 64-entry batch at a time at 8 fixed points of the loop (between load issues), and item i-1's
// fixed store sequence goes out at the end of item i.  Same entries, same lists, same bits.
// ------------------------------------------------------------------------------------------
#ifndef FLC_DS2_CAP
#define FLC_DS2_CAP 384              // k_ds_filter2 staging capacity per item (4.7 %; C4 items hold ~2.3 %)
#endif
#ifndef FLC_DS2_WPE
#define FLC_DS2_WPE 5                // LDS: 32 KB per block (FLC_DS2_CAP 384), 5 blocks per CU
#endif
template <int RING, int GCAP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FLC_DS2_WPE))) void k_ds_filter2(RowSrc rows, int64_t n, int64_t r0, int64_t rn, int64_t rb, int64_t d, DsWs ws, UniformSrc) {
    constexpr int FGS = DS_FGS, NH = DS_NH;
    // GCAP: the staging capacity (candidates per item; more -> the row is folded dense), at most
    // DS_GCAP, the stride of the items' ambiguous-entry regions
    static_assert(FGS == 2 && NH == 4 && GCAP % 128 == 0 && GCAP <= DS_GCAP && DS_HCAP == 128, "batch points / copy-out layout");
    static_assert(16 % RING == 0, "ring must divide the 16 loads of a chunk");
    constexpr int NB = GCAP / 64;                          // classification batches of one item
    constexpr int DS_ITEM_STORES = 4 + GCAP / 128;          // partial, itm, tab, sure and ambiguous copy-outs
    __shared__ __attribute__((aligned(16))) uint2 stage[2][4][GCAP + 64];
    __shared__ __attribute__((aligned(16))) uint16_t stage16[4][NH * DS_HCAP];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t G = ws.G;
    const int64_t items = rn * G;
    const int64_t stride = (int64_t)gridDim.x * 4;
    int64_t it = (int64_t)blockIdx.x * 4 + wv;
    if (it >= items) return;
    const uint32_t lphi = (uint32_t)lane * 0x9E3779B1u;    // group index g = c*1024 + 64 L + lane
    uint16_t* s16 = stage16[wv];
    float4 ring[RING];
    auto item_at = [&](int64_t t, int64_t& r, int64_t& g) {   // k_ds_filter's item order
        const int64_t blk = t / (rb * G), rem = t - blk * rb * G;
        const int64_t bn = min(rb, rn - blk * rb);
        g = rem / bn;
        r = r0 + blk * rb + (rem - g * bn);
    };
    int64_t row, gi0;
    item_at(it, row, gi0);
    int64_t c = gi0 * FGS;
    auto rs = chunk_rsrc(rows.row_s(row), c * CHUNK, d);
#pragma unroll
    for (int L = 0; L < RING - 1; ++L) {
        ring[L] = load_q(rs, lane, L);
        __builtin_amdgcn_sched_barrier(0);
    }
    {
        const auto nd = __builtin_amdgcn_make_buffer_rsrc(ws.enta, (short)0, 0, 0x00020000);
#pragma unroll
        for (int k = 0; k < DS_ITEM_STORES; ++k) __builtin_amdgcn_raw_buffer_store_b32(0u, nd, lane * 4, k * 256, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
    // the previous item (pv): its row, item, candidate count, norm partial, classification scales
    bool pv = false, pfits = true;
    int64_t prow = 0, pgi = 0;
    uint32_t pncl = 0, prk = 0;
    double pa2 = 0.0;
    float pq0 = 0.f, pq1 = 0.f;
    uint32_t hs[NH], na = 0;                               // its classification counters
#pragma unroll
    for (int u = 0; u < NH; ++u) hs[u] = 0;
    int par = 0;
    // batch b of the previous item's candidates: sure entries to s16 (half h's at h * DS_HCAP),
    // ambiguous ones compacted in place in its staging (a batch reads its 64 slots before it
    // writes lower ones); k_ds_filter's classification, verbatim
    auto classify = [&](int b) {
        uint2* sgp = stage[par ^ 1][wv];
        const uint32_t e = (uint32_t)(b * 64 + lane);
        const bool v = e < pncl;
        const uint2 en = v ? sgp[e] : make_uint2(0u, 0u);
        const float x = __uint_as_float(en.y), ax = fabsf(x);
        const uint32_t loc = en.x & 0x1FFFu;
        const uint32_t j0 = (uint32_t)(pgi * (FGS * CHUNK));
        const uint32_t hi8 = ds_hi8(j0 + loc, prk);
        const uint32_t h24 = (hi8 << 16) | (fmix32(colbase(j0 + loc) + (prk ^ 0x27D4EB2Fu)) >> 16);   // h >> 8
        const float hf = (float)h24 * 0x1p-24f, hfu = (float)(h24 + 1u) * 0x1p-24f;
        const bool inl = ax * pq0 <= 1.0f - 0x1p-18f;
        const bool nz = v && !(x == 0.f);
        const bool sure = nz && inl && fmaf(ax, pq1, hf) >= 1.0f + 0x1p-20f;
        const bool drop = !nz || (inl && fmaf(ax, pq0, hfu) < 1.0f - 0x1p-20f);
        const bool amb = !sure && !drop;
        const uint32_t u = loc >> 11;
        uint32_t pin = 0;
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            const uint64_t mh = __ballot(sure && u == (uint32_t)h);
            const uint32_t ph = __builtin_amdgcn_mbcnt_hi((uint32_t)(mh >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mh, hs[h]));
            pin = u == (uint32_t)h ? ph : pin;
            hs[h] += (uint32_t)__popcll(mh);
        }
        if (sure && pin < (uint32_t)DS_HCAP)
            s16[u * DS_HCAP + pin] = (uint16_t)((loc & (HCHUNK - 1)) | ((en.y >> 31) << 11) | (1u << 12));
        const uint64_t ma = __ballot(amb);
        const uint32_t pa = __builtin_amdgcn_mbcnt_hi((uint32_t)(ma >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ma, na));
        if (amb) sgp[pa] = make_uint2(loc | (hi8 << 13), en.y);     // k_ds_resolve's entry
        na += (uint32_t)__popcll(ma);
    };
    // the previous item's stores: k_ds_filter's fixed sequence, every store a range-checked buffer
    // store (no previous item: all dropped), so the vmcnt queue has the same shape every time
    auto finish = [&]() {
        bool ovf = !pfits;
#pragma unroll
        for (int u = 0; u < NH; ++u) ovf |= hs[u] > (uint32_t)DS_HCAP;
        typedef unsigned int u2v __attribute__((ext_vector_type(2)));
        typedef unsigned int u4v __attribute__((ext_vector_type(4)));
        {
            const auto od = __builtin_amdgcn_make_buffer_rsrc(ws.partial + prow * G + pgi, (short)0, pv ? 8 : 0, 0x00020000);
            const uint64_t ab = __builtin_bit_cast(uint64_t, pa2);
            const u2v v2 = {(unsigned)ab, (unsigned)(ab >> 32)};
            __builtin_amdgcn_raw_buffer_store_b64(v2, od, 0, 0, 0);
        }
        {
            const auto od = __builtin_amdgcn_make_buffer_rsrc(ws.itm + pgi * n + prow, (short)0, pv ? 4 : 0, 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b32(ovf ? DS_OVF : na, od, 0, 0, 0);
        }
        {
            // halves past the row end land in the tab's padding rows (G * NH >= H)
            const uint32_t u = (uint32_t)lane & (NH - 1);
            uint32_t hc = 0;
#pragma unroll
            for (int v = 0; v < NH; ++v) hc = (uint32_t)v == u ? hs[v] : hc;
            const auto od = __builtin_amdgcn_make_buffer_rsrc(ws.tabs + pgi * NH * n + prow, (short)0,
                                                              pv ? (int)(((NH - 1) * n + 1) * 8) : 0, 0x00020000);
            const u2v v2 = {0u, ovf ? 0u : hc};
            __builtin_amdgcn_raw_buffer_store_b64(v2, od, u * (uint32_t)n * 8u, 0, 0);
        }
        {
            const uint32_t u = (uint32_t)lane >> 4, k8 = ((uint32_t)lane & 15u) * 8u;
            uint32_t hc = 0;
#pragma unroll
            for (int v = 0; v < NH; ++v) hc = (uint32_t)v == u ? hs[v] : hc;
            const bool put = pv && !ovf && k8 < hc;
            const uint32_t hstride = (uint32_t)n * (DS_HCAP * 2);               // bytes
            const auto od = __builtin_amdgcn_make_buffer_rsrc(ws.ent16 + (pgi * NH * n + prow) * DS_HCAP, (short)0,
                                                              (int)((NH - 1) * hstride + DS_HCAP * 2), 0x00020000);
            const uint4 v = reinterpret_cast<const uint4*>(s16)[lane];
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, v), od, put ? u * hstride + k8 * 2u : 0x7FFFFFF0u, 0, 0);
        }
        {
            const uint32_t nrec = (pv && !ovf) ? ((na + 1u) & ~1u) * 8u : 0u;
            const auto od = __builtin_amdgcn_make_buffer_rsrc(ws.enta + prow * ws.cap + pgi * DS_GCAP, (short)0, (int)nrec, 0x00020000);
            const uint4* sq = reinterpret_cast<const uint4*>(stage[par ^ 1][wv]);
#pragma unroll
            for (int k = 0; k < GCAP / 128; ++k) {
                const uint4 v = sq[k * 64 + lane];
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, v), od, (k * 64 + lane) * 16, 0, 0);
            }
        }
    };
    while (it < items) {
        const float qc = sload(ws.qc + row);
        const uint32_t rk = sload(ws.rk + row);
        const int64_t gi = c / FGS;
        const int64_t nit = it + stride;
        uint32_t cnt = 0;
        double a2 = 0.0;
        int64_t nrow = row, nc = c;
        const uint32_t sla = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(__attribute__((address_space(3))) uint2*)stage[par][wv]);
        na = 0;
#pragma unroll
        for (int u = 0; u < NH; ++u) hs[u] = 0;
#pragma unroll
        for (int sub = 0; sub < FGS; ++sub, ++c) {
            const int64_t j0 = c * CHUNK;
            __amdgpu_buffer_rsrc_t rsn;
            if (sub + 1 < FGS) {
                rsn = chunk_rsrc(rows.row_s(row), j0 + CHUNK, d);
            } else if (nit < items) {
                int64_t ngi;
                item_at(nit, nrow, ngi);
                nc = ngi * FGS;
                rsn = chunk_rsrc(rows.row_s(nrow), nc * CHUNK, d);
            } else {
                rsn = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(rows.row_s(row)), (short)0, 0, 0x00020000);
            }
            uint32_t jb = (uint32_t)lane * 4u + (uint32_t)sub * CHUNK;
            asm volatile("" : "+v"(jb));
            const uint32_t gb = lphi + (uint32_t)(c * 1024) * 0x9E3779B1u + rk;
#pragma unroll
            for (int L = 0; L < 16; ++L) {
                const int P = L + RING - 1;
                ring[P % RING] = P < 16 ? load_q(rs, lane, P) : load_q(rsn, lane, P - 16);
                const float4 x = ring[L % RING];
                const uint32_t hg = gmix(gb + (uint32_t)(L * 64) * 0x9E3779B1u);
                const float vq[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    a2 = fma((double)vq[q], (double)vq[q], a2);
                    const float hi = (float)((hg >> (8 * q)) & 0xFFu);
                    const bool f = fmaf(fabsf(vq[q]), qc, hi) > DS_QT;
                    const uint64_t m = __ballot(f);
                    if (f) {
                        const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                        uint32_t sb = sla + min(cnt, (uint32_t)GCAP) * 8u;
                        asm volatile("" : "+s"(sb));
                        const uint32_t la = sb + pre * 8u;
                        asm volatile("ds_write2_b32 %0, %1, %2 offset1:1" ::"v"(la), "v"(jb + (uint32_t)(L * 256 + q)),
                                     "v"(__float_as_uint(vq[q])) : "memory");
                    }
                    cnt += (uint32_t)__popcll(m);
                }
                asm volatile("" : "+v"(a2));
                // the previous item's batches, between load issues (8 points cover GCAP)
                if ((L & 3) == 1) {
                    const int b = sub * 4 + (L >> 2);
                    if ((uint32_t)(b * 64) < pncl) classify(b);
                }
            }
            rs = rsn;
        }
        a2 = wave_sum(a2);
        finish();
        prow = row; pgi = gi; pfits = cnt <= GCAP; pncl = pfits ? cnt : 0u; pa2 = a2; prk = rk;
        pq0 = sload(ws.q0 + row); pq1 = sload(ws.q1 + row);
        pv = true;
        // the copy-out reads and the classification precede the next item's staging writes
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        par ^= 1;
        it = nit;
        row = nrow;
        c = nc;
    }
    // the last item: classify, then its stores
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    na = 0;                                                  // (its staging: buffer par ^ 1)
#pragma unroll
    for (int u = 0; u < NH; ++u) hs[u] = 0;
    for (int b = 0; b < NB; ++b)
        if ((uint32_t)(b * 64) < pncl) classify(b);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    finish();
}

// ------------------------------------------------------------------------------------------
// Norm and row mode: one wave per row.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_ds_final(int64_t r0, int64_t rn, DsWs ws, const float* __restrict__ w,
                                                  float* __restrict__ pnorm_out) {
    const int lane = threadIdx.x & 63;
    const int64_t row = r0 + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= r0 + rn) return;
    double a = 0.0;
    uint32_t ov = 0;
    int64_t k = lane;
    for (; k + 7 * 64 < ws.G; k += 8 * 64) {                 // 8 far loads per round trip, same order
        double v[8];
        uint32_t t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) { v[u] = ws.partial[row * ws.G + k + u * 64]; t[u] = ws.itm[(k + u * 64) * ws.n + row]; }
#pragma unroll
        for (int u = 0; u < 8; ++u) { a += v[u]; ov |= t[u] == DS_OVF; }
    }
    for (; k < ws.G; k += 64) { a += ws.partial[row * ws.G + k]; ov |= ws.itm[k * ws.n + row] == DS_OVF; }
    a = wave_sum(a);
    ov = __ballot(ov != 0u) != 0ull;
    if (lane == 0) {
        const float nv = (float)sqrt(a);
        ws.pn[row] = nv;
        if (pnorm_out) pnorm_out[row] = nv;
        ws.rpn[row] = 1.0f / nv;
        uint32_t fl = ws.flags[row];
        const bool wbad = w && !(fabsf(w[row]) <= 3.4028235e38f);
        if (!(nv >= ws.nlo[row]) || !(nv <= ws.nhi[row]) || !(nv <= 3.4028235e38f) || ov || wbad) fl |= DS_DENSE;
        if (nv >= 0x1p-40f && nv <= 0x1p80f) fl |= DS_FAST;   // |x| / norm may use div_fast
        ws.flags[row] = fl;
    }
}

// Row state of the exact encode (wave-uniform).
struct DsRow {
    float n, rn;          // norm, RN(1 / norm)
    uint32_t rk2;         // row key of the low draw: rk ^ 0x27D4EB2F (common.hpp dev_draw)
    bool fast;            // norm inside the div_fast window
};

// The level C(x)_j of standard dithering (compressors.py:270-299) picks for one element, exactly as
// DitherOp::apply<false> (codec_ops.hpp) computes it: the draw's top byte comes with the entry
// (hi8), and the rare slow cases (|x| or a level gap outside the fast-division window, the
// interval guess off by one) are taken behind wave-level branches instead of being if-converted.
// Returns the level's value (0 outside every interval) and index (-1 there).
struct DsLev {
    float v;
    int idx;
};
// COMPAT: the draw is the caller's float64 uniform ud, against p = p2 * 2^-32 as DitherOp<.., true>.
template <bool COMPAT>
__device__ inline DsLev ds_level(float x, uint32_t j, uint32_t hi8, double ud, const DsRow& r, const float4* tab, int s,
                                 float sf) {
    const float ax = fabsf(x);
    FastDiv dn;
    dn.b = r.n; dn.rb = r.rn; dn.ok = true;
    float y = div_fast(ax, dn);                                   // |x| / pnorm
    const bool slow = !(r.fast && (ax >= 0x1p-80f || ax == 0.f) && ax <= 0x1p80f);
    if (__builtin_expect(__ballot(slow) != 0ull, 0)) {
        if (slow) y = ax / r.n;
    }
    int g = (int)(y * sf);                                        // y >= 0; NaN -> 0
    g = g > s - 1 ? s - 1 : g;
    float4 t = tab[g];
    const bool off = (y < t.x) | (y > t.y);
    if (__builtin_expect(__ballot(off) != 0ull, 0)) {            // std levels RN(k/s): at most one off
        if (off) {
            g = (y < t.x) ? (g > 0 ? g - 1 : 0) : (g < s - 1 ? g + 1 : g);
            t = tab[g];
        }
    }
    const bool in = y <= t.y;                                     // y > 1 or NaN: no interval -> 0
    const float num = y - t.y;
    FastDiv dd;
    dd.b = t.z; dd.rb = t.w; dd.ok = true;
    float p2 = div_fast(num, dd);                                 // p * 2^32
    const bool gap_slow = t.w == 0.f;                             // gap outside the window (load_table)
    if (__builtin_expect(__ballot(gap_slow) != 0ull, 0)) {
        if (gap_slow) p2 = num / t.z;
    }
    bool down;
    if constexpr (COMPAT) {
        down = ud < (double)ldexpf(p2, -32);
    } else {
        uint32_t thr;
        asm("v_cvt_u32_f32 %0, %1" : "=v"(thr) : "v"(ceilf(p2)));   // saturating: thr32(p)
        // draw h = hi8 << 24 | lo24 against thr: the top byte decides unless it equals thr's (1 in
        // 256), so the low hash is computed only for those lanes
        const uint32_t th = thr >> 24;
        down = hi8 < th;
        const bool tie = hi8 == th;
        if (__builtin_expect(__ballot(tie) != 0ull, 0)) {
            if (tie) down = ((hi8 << 24) | (fmix32(colbase(j) + r.rk2) >> 8)) < thr;
        }
    }
    DsLev l;
    l.v = in ? (down ? t.x : t.y) : 0.f;
    l.idx = in ? (down ? g : g + 1) : -1;
    return l;
}

// C(x)_j: (lev * sign(x)) * pnorm
template <bool COMPAT>
__device__ inline float ds_encode(float x, uint32_t j, uint32_t hi8, double ud, const DsRow& r, const float4* tab, int s,
                                  float sf) {
    const DsLev l = ds_level<COMPAT>(x, j, hi8, ud, r, tab, s, sf);
    return (x == 0.f) ? 0.f : copysignf(l.v, x) * r.n;
}


// ------------------------------------------------------------------------------------------
// Resolve: one wave per 64 filter items — item gi of 64 consecutive rows, one lane each, so the
// per-item tables ([item][row]) are read and written coalesced; their ambiguous candidates,
// spread over the wave's lanes, encoded with their rows' norms; the nonzero ones appended as list
// entries after the sure entries of their half chunk (an LDS counter per (item, half): the order
// inside one row's list is free, its columns are distinct), the counts into cntr.  A level above
// DS_MAXLEV or a full half region turns the row dense.
// ------------------------------------------------------------------------------------------
template <bool COMPAT>
__global__ __launch_bounds__(256) void k_ds_resolve(int64_t n, int64_t r0, int64_t rn, DsWs ws,
                                                    const float* __restrict__ levels, int s, UniformSrc us) {
    constexpr int NH = DS_NH;
    __shared__ __attribute__((aligned(16))) float4 tab[DS_MAXS];
    __shared__ uint32_t pre[4][65], irow[4][64], igi[4][64], ikey[4][64], imode[4][64], cs[4][64][NH], cr[4][64][NH];
    __shared__ float ipn[4][64], irpn[4][64];
    __shared__ int own[4][64];
    load_table(levels, s, tab);
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const float sf = (float)s;
    const int64_t nrb = (rn + 63) / 64, groups = nrb * ws.G;
    for (int64_t grp = (int64_t)blockIdx.x * 4 + wv; grp < groups; grp += (int64_t)gridDim.x * 4) {
        const uint32_t gi = (uint32_t)(grp / nrb);
        const int64_t row = r0 + (grp - (int64_t)gi * nrb) * 64 + lane;
        const bool valid = row < r0 + rn;
        uint32_t na = 0, mode = DS_DENSE;
        if (valid) {
            mode = ws.flags[row];
            if (!(mode & DS_DENSE)) na = ws.itm[(int64_t)gi * n + row];
        }
        // exclusive prefix of na over the lanes
        uint32_t inc = na;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(inc, o, 64);
            inc += lane >= o ? t : 0u;
        }
        const uint32_t total = __shfl(inc, 63, 64);
        pre[wv][lane] = inc - na;
        if (lane == 0) pre[wv][64] = total;
        irow[wv][lane] = (uint32_t)row;
        igi[wv][lane] = gi;
        ikey[wv][lane] = (valid ? ws.rk[row] : 0u) ^ 0x27D4EB2Fu;
        imode[wv][lane] = mode;
        ipn[wv][lane] = valid ? ws.pn[row] : 1.f;
        irpn[wv][lane] = valid ? ws.rpn[row] : 1.f;
#pragma unroll
        for (int u = 0; u < NH; ++u) {
            cs[wv][lane][u] = (na > 0u) ? ws.tabs[((int64_t)gi * NH + u) * n + row].y : 0u;
            cr[wv][lane][u] = 0u;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        // The candidates of the 64 items, flattened: slot t belongs to the last lane k with
        // pre[k] <= t.  Per window of 64 slots the owners come from marks (lane k with candidates
        // writes its lane id at slot pre[k] - t0) and a max-scan over the lanes (owners rise with
        // the slot), slots before the window's first mark taking the previous window's last owner;
        // the next window's owners and candidate loads are issued before this window is encoded.
        const uint32_t mypre = inc - na;
        uint32_t carry = 0;
        auto owner = [&](uint32_t t0) -> uint32_t {
            own[wv][lane] = -1;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            if (na > 0u && mypre >= t0 && mypre < t0 + 64u) own[wv][mypre - t0] = lane;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            int v = own[wv][lane];
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int w = __shfl_up(v, o, 64);
                v = (lane >= o && w > v) ? w : v;
            }
            const uint32_t k = v < 0 ? carry : (uint32_t)v;
            carry = __shfl(k, 63, 64);
            return k;
        };
        auto fetch = [&](uint32_t t0, uint32_t k) -> uint2 {
            const uint32_t t = t0 + (uint32_t)lane;
            const uint32_t e = t - pre[wv][k];
            const int64_t ei = t < total ? (int64_t)irow[wv][k] * ws.cap + (int64_t)igi[wv][k] * DS_GCAP + e : 0;
            const uint2 v = ws.enta[ei];                          // lanes past the total: entry 0 (ignored)
            return v;
        };
        // The first RW windows' owners and candidate loads are all issued before any is encoded
        // (their gathers from 64 rows' regions overlap instead of costing one round trip each);
        // windows past RW are fetched one ahead.
        constexpr int RW = FLC_DS_RW;
        uint32_t kw[RW];
        uint2 ew[RW];
#pragma unroll
        for (int w = 0; w < RW; ++w) {
            kw[w] = 0u;
            ew[w] = make_uint2(0u, 0u);
            if ((uint32_t)w * 64u < total) { kw[w] = owner((uint32_t)w * 64u); ew[w] = fetch((uint32_t)w * 64u, kw[w]); }
        }
        uint32_t kc = 0;
        uint2 enc = make_uint2(0u, 0u);
        if ((uint32_t)RW * 64u < total) { kc = owner((uint32_t)RW * 64u); enc = fetch((uint32_t)RW * 64u, kc); }
        for (uint32_t t0 = 0; t0 < total; t0 += 64) {
            const uint32_t t = t0 + (uint32_t)lane;
            const bool tv = t < total;
            const uint32_t wi = t0 >> 6;
            uint32_t k = kc;
            uint2 en = enc;
            if (wi < (uint32_t)RW) {
#pragma unroll
                for (int w = 0; w < RW; ++w)
                    if ((uint32_t)w == wi) { k = kw[w]; en = ew[w]; }
            } else if (t0 + 64u < total) {
                const uint32_t kn = owner(t0 + 64u);
                const uint2 nn = fetch(t0 + 64u, kn);
                k = kc; en = enc;
                kc = kn; enc = nn;
            }
            en = tv ? en : make_uint2(0u, 0u);
            const int64_t rk_ = irow[wv][k];
            const uint32_t gk = igi[wv][k];
            const float x = __uint_as_float(en.y);
            const uint32_t loc = en.x & 0x1FFFu;
            DsRow rr;
            rr.n = ipn[wv][k];
            rr.rn = irpn[wv][k];
            rr.rk2 = ikey[wv][k];
            rr.fast = (imode[wv][k] & DS_FAST) != 0u;
            const uint32_t j = gk * (uint32_t)(DS_FGS * CHUNK) + loc;
            double ud = 0.0;                                  // compat: the element's uniform
            if constexpr (COMPAT) ud = us.u[(tv ? rk_ : 0) * us.uld + (tv ? j : 0u)];
            const DsLev l = ds_level<COMPAT>(x, j, en.x >> 13, ud, rr, tab, s, sf);
            const bool keep = tv && !(x == 0.f) && l.idx > 0 && !(l.v == 0.f);
            if (keep) {
                const uint32_t u = loc >> 11;
                const uint32_t slot = atomicAdd(&cr[wv][k][u], 1u);
                const uint32_t pos = cs[wv][k][u] + slot;
                if (l.idx > DS_MAXLEV || pos >= (uint32_t)DS_HCAP) {
                    atomicOr(&ws.flags[rk_], DS_DENSE);
                } else {
                    ws.ent16[(((int64_t)gk * NH + u) * n + rk_) * DS_HCAP + pos] =
                        (uint16_t)((loc & (HCHUNK - 1)) | ((en.y >> 31) << 11) | ((uint32_t)l.idx << 12));
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (valid && na > 0u) {
#pragma unroll
            for (int u = 0; u < NH; ++u) ws.cntr[((int64_t)gi * NH + u) * n + row] = cr[wv][lane][u];
        } else if (valid) {
#pragma unroll
            for (int u = 0; u < NH; ++u) ws.cntr[((int64_t)gi * NH + u) * n + row] = 0u;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
}

// ------------------------------------------------------------------------------------------
// Chunk-owner fold.  One wave per half chunk, fp32 LDS tile, rows in order; per row its list
// (sure + resolved entries: copysign(levels[level], sign) * norm) — the first 64 entries from a
// ring of AP rows in flight, the rest read in place — or, for DENSE rows, the half chunk of x
// itself, encoded.  Contributions are W ? w_i * C(x)_j : C(x)_j.
// ------------------------------------------------------------------------------------------
struct DsMeta {
    uint32_t off, cnt;
    float pn, rpn, w;
    uint32_t rk, mode;
};

__device__ inline DsMeta ds_meta(const DsWs& ws, int64_t c, int64_t n, int64_t rend, int64_t r, const float* w) {
    DsMeta m;
    m.off = 0; m.cnt = 0;
    m.pn = 1.f; m.rpn = 1.f; m.w = 1.f; m.rk = 0; m.mode = 0;
    if (r < rend) {
        // every load issued at once (no flags -> tab dependency): a dense row's count is dropped below
        m.pn = ws.pn[r];
        m.rpn = ws.rpn[r];
        m.rk = ws.rk[r];
        m.mode = ws.flags[r];
        const uint32_t c0 = ws.tabs[c * n + r].y, c1 = ws.cntr[c * n + r];   // c: half-chunk index
        m.cnt = (m.mode & DS_DENSE) ? 0u : c0 + c1;
        if (w) m.w = w[r];
    }
    return m;
}

// ds_meta without anything computed from the loads: off = sure entries, cnt = resolved entries
// (their sum is the list length of a non-dense row), mode = the row's flags
__device__ inline DsMeta ds_meta_raw(const DsWs& ws, int64_t c, int64_t n, int64_t rend, int64_t r, const float* w) {
    DsMeta m;
    m.off = 0; m.cnt = 0;
    m.pn = 1.f; m.rpn = 1.f; m.w = 1.f; m.rk = 0; m.mode = 0;
    if (r < rend) {
        m.pn = ws.pn[r];
        m.rpn = ws.rpn[r];
        m.rk = ws.rk[r];
        m.mode = ws.flags[r];
        m.off = ws.tabs[c * n + r].y;
        m.cnt = ws.cntr[c * n + r];
        if (w) m.w = w[r];
    }
    return m;
}

#ifndef FLC_DS_MASKLD
#define FLC_DS_MASKLD 0
#endif
#ifndef FLC_DS_L1REG
#define FLC_DS_L1REG 0               // k_ds_accum (FLC_DS_WIDE): level-1 value from a register
#endif
#ifndef FLC_DS_LDSADD
#define FLC_DS_LDSADD 0              // k_ds_accum (FLC_DS_WIDE): tile updates as LDS fp32 adds
#endif
#ifndef FLC_DS_WIDE
#define FLC_DS_WIDE 1                // k_ds_accum (with FLC_DS_RAWRING): 64-row batches of list windows by LDS DMA
                                     // (round 5: the fold 0.93 -> 0.70-0.73 ms per C4 step, step -0.05 ms, same
                                     // allocation, profiles/r05/ab_c4_fold.txt)
#endif
#ifndef FLC_DS_RAWRING
#define FLC_DS_RAWRING 1             // k_ds_accum: raw list loads, masked where folded (the fast loop below)
#endif
#ifndef FLC_DS_AW
#define FLC_DS_AW 1                  // waves per fold workgroup (LDS: one 8 KB tile per wave)
#endif
constexpr int DS_AW = FLC_DS_AW;
#ifndef FLC_DS_AWPE
#define FLC_DS_AWPE 0                // k_ds_accum: minimum waves per SIMD the register allocation targets (0: compiler's choice)
#endif
#if FLC_DS_WIDE
// the compiler's occupancy model of the 16 KB of LDS per wave gives up on any waves-per-EU target
// (it then takes 400 registers): cap the registers explicitly (4 waves per SIMD: 128)
#define FLC_DS_ACCUM_ATTR __attribute__((amdgpu_num_vgpr(128)))
#elif FLC_DS_AWPE > 0
#define FLC_DS_ACCUM_ATTR __attribute__((amdgpu_waves_per_eu(FLC_DS_AWPE)))
#else
#define FLC_DS_ACCUM_ATTR
#endif

// Folds rows [r0, r0 + rn) into the running sums: the first group starts the tiles at -0, the others
// continue from `part` (the previous group's tiles); the last group resolves untouched columns
// over ALL n rows and writes out = sums / wt, the others write their tiles back to `part`.
// Small workgroups with only the tile in LDS (the dense rows' level table is ws.gtab): up to 19
// waves per CU for this latency-bound walk (a 4-wave block with the table in LDS fit 3 per CU).
// The row walk is a ring of AP rows' first 64 entries: row q's slot is refilled with row q + AP
// as soon as q is folded, so a list load has AP - 1 rows of work in front of it.
template <bool W, int AP, bool COMPAT>
__global__ __launch_bounds__(64 * DS_AW) FLC_DS_ACCUM_ATTR void k_ds_accum(RowSrc rows, int64_t n, int64_t r0, int64_t rn, int first, int last,
                                                  int64_t d, DsWs ws, const float* __restrict__ levels, int s,
                                                  const float* __restrict__ w, float wt, float* __restrict__ part,
                                                  float* __restrict__ out, UniformSrc us) {
    static_assert(64 % AP == 0, "row groups tile the 64-row batch");
    constexpr uint32_t NONE = 0xFFFFFFFFu;
    __shared__ __attribute__((aligned(16))) float tile[DS_AW][HCHUNK];
    __shared__ __attribute__((aligned(16))) uint16_t dstg[DS_AW][FLC_DS_WIDE ? 8 : 1][FLC_DS_WIDE ? 512 : 1];   // FLC_DS_WIDE: 8 KB per wave
    __shared__ float lvl[DS_MAXLEV + 1];
    if (threadIdx.x <= (unsigned)DS_MAXLEV) lvl[threadIdx.x] = (int)threadIdx.x <= s ? levels[threadIdx.x] : 0.f;
    __syncthreads();
    const float4* tab = ws.gtab;
    const int lane = threadIdx.x & 63;
    const int wv = DS_AW == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t H = nhalves(d);
    float* tl = tile[wv];
    const int64_t rend = r0 + rn;
    const int64_t nb = (rn + 63) / 64;
    const float sf = (float)s;
    for (int64_t h = (int64_t)blockIdx.x * DS_AW + wv; h < H; h += (int64_t)gridDim.x * DS_AW) {
        // The tile starts at -0.0: (-0) + t == t for every nonzero t, and a column that received a
        // nonzero contribution never returns to -0 (x + y == -0 needs two -0 addends), so a final
        // -0 bit pattern marks exactly the untouched columns.  Zero contributions are not added.
        // Adds are read-modify-writes of the wave's own tile, in row order (one wave executes its
        // LDS operations in program order; the lanes of one instruction hit distinct columns), so
        // each column sees its rows' terms in row order.
        const uint32_t hbase = (uint32_t)(h * HCHUNK);
        const int64_t len = min((int64_t)HCHUNK, d - (int64_t)hbase);
        if (FLC_TILE_V4 && !first && len == HCHUNK) {
            // the carried tile with every load in flight at once (the loop of load -> LDS write
            // pairs below waits one memory latency per 64 columns: 32 per tile)
            const float4* p4 = reinterpret_cast<const float4*>(part + hbase);
            float4 v[HCHUNK / 256];
#pragma unroll
            for (int k = 0; k < HCHUNK / 256; ++k) v[k] = p4[k * 64 + lane];
#pragma unroll
            for (int k = 0; k < HCHUNK / 256; ++k) reinterpret_cast<float4*>(tl)[k * 64 + lane] = v[k];
        } else {
            for (int i = lane; i < HCHUNK; i += 64) tl[i] = (first || i >= len) ? -0.f : part[hbase + i];
        }
        DsMeta cur = ds_meta(ws, h, n, rend, r0 + lane, w), nxt;
        uint32_t ra[AP];                        // ring: first 64 entries of rows q .. q + AP - 1
        // a list's 64-entry window never leaves its item's half region (DS_HCAP >= 64): loaded
        // whole, lanes past the count dropped; an empty list (rows past the end, dense rows) reads
        // the array's first 64 entries instead
        auto fetch = [&](const DsMeta& m, int q, int64_t row, int slot) {
            const uint32_t cnt = __builtin_amdgcn_readlane(m.cnt, q);
            const uint16_t* p = cnt ? ws.ent16 + (h * n + row) * DS_HCAP : ws.ent16;
#if FLC_DS_MASKLD
            // only the lanes of the list's entries load (the region is 256 B, a list ~80 B)
            uint32_t v = NONE;
            if ((uint32_t)lane < cnt) v = __builtin_nontemporal_load(p + lane);
            ra[slot] = v;
#else
            const uint32_t v = p[lane];
            ra[slot] = (uint32_t)lane < cnt ? v : NONE;
#endif
        };
        // (LDS float atomic adds instead of the read-modify-write — one wave's LDS operations run
        // in issue order, so the row order would hold — measured 1.34 against 0.51 ms at C4)
        auto add = [&](uint32_t loc, float t) {
            if (!(t == 0.f)) tl[loc] = tl[loc] + t;
        };
        auto value = [&](uint32_t e, float pn) {            // copysign(levels[lev], sign) * pnorm
            const float lv = lvl[(e >> 12) & 15u];
            return __uint_as_float(__float_as_uint(lv) | ((e & 0x800u) << 20)) * pn;
        };
        auto row_state = [&](const DsMeta& m, int q, float& pn, float& wi) {
            pn = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(m.pn), q));
            wi = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(m.w), q));
        };
        // refill the slot of row q (this batch) with row q + AP (past the batch end: the next
        // batch's meta; past n: empty lists)
        auto refill = [&](int q, int64_t i0) {
            if (q + AP < 64) fetch(cur, q + AP, i0 + q + AP, q % AP);
            else fetch(nxt, q + AP - 64, i0 + q + AP, q % AP);   // q % AP: static once unrolled
        };
#if FLC_DS_RAWRING
        // Raw ring: row q's slot holds the first 64 u16 of its region, loaded whatever its count
        // (rows clamped to the array's last row) and masked with the count where the row is
        // folded.  The refill address thus needs no row state, and no select sits between a load
        // and its use: each row waits for its own load only (a static vmcnt(AP - 1)).  (The
        // previous form masked at the load and took a general path inside the same loop: the
        // compiler copied the ring at the back-edges and waited for the whole ring there.)
        int64_t b = 0;
#if FLC_DS_WIDE
        cur = ds_meta_raw(ws, h, n, rend, r0 + lane, w);
        const float lv1 = lvl[1];
        // Wide batches through LDS DMA: a 64-row batch's list windows (the first 128 B of each row's
        // region) are 8 loads of 16 B per lane straight into the wave's 8 KB staging (lane l: row
        // l / 8 of its 8-row slot, bytes 16 (l % 8) ..; no ring registers), issued a whole batch
        // ahead.  The compiler waits for every outstanding load before the first staging read
        // (vmcnt(0): it does not track LDS DMA per slot), so each batch reads all its 64 entries
        // per lane first, then issues the next batch's 8 loads and its row state, then folds the
        // 64 rows: each batch's loads have a whole batch of folding to arrive in (the 16-row
        // register ring waited a memory latency every 16 rows).
        auto dma = [&](int64_t row0, int sl) {
            const uint16_t* src = ws.ent16 + (h * n + min(row0 + (lane >> 3), n - 1)) * DS_HCAP + (lane & 7) * 8;
            __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)&dstg[wv][sl][0], 16, 0, 0);
        };
#pragma unroll
        for (int sl = 0; sl < 8; ++sl) dma(r0 + 8 * sl, sl);
        for (; b < nb; ++b) {
            const int64_t i0 = r0 + b * 64;
            if (__ballot((cur.mode & DS_DENSE) != 0u) != 0ull) break;
            // rows with more than 64 entries in this half (~1e-4 of C4's): the batch takes the rolled
            // path below, which reads the rest of their lists directly
            const uint64_t lng = __ballot(cur.off + cur.cnt > 64u);
            if (__builtin_expect(lng == 0ull, 1)) {
                // the batch's 64 entries of this lane, two rows per register
                uint32_t ent2[32];
#pragma unroll
                for (int q = 0; q < 64; q += 2)
                    ent2[q >> 1] = (uint32_t)dstg[wv][q >> 3][(q & 7) * 64 + lane] |
                                   ((uint32_t)dstg[wv][(q + 1) >> 3][((q + 1) & 7) * 64 + lane] << 16);
                __builtin_amdgcn_s_waitcnt(0xC07F);                  // lgkmcnt(0): the slots are read
                // the next batch's row state, raw (nothing computed from it before the next batch: a
                // use here would wait for the loads behind it), then its list windows
                nxt = ds_meta_raw(ws, h, n, rend, i0 + 64 + lane, w);
#pragma unroll
                for (int sl = 0; sl < 8; ++sl) dma(i0 + 64 + 8 * sl, sl);
#pragma unroll
                for (int q = 0; q < 64; ++q) {
                    // rows in order; the scheduler does not hoist 64 rows' work (register pressure)
                    __builtin_amdgcn_sched_barrier(0);
                    float pn, wi;
                    row_state(cur, q, pn, wi);
                    // (no dense row in the batch: the count is the sure + resolved entries)
                    const uint32_t cnt = __builtin_amdgcn_readlane(cur.off, q) + __builtin_amdgcn_readlane(cur.cnt, q);
                    const uint32_t raw = (q & 1) ? (ent2[q >> 1] >> 16) : (ent2[q >> 1] & 0xFFFFu);
                    const uint32_t a = (uint32_t)lane < cnt ? raw : NONE;
#if FLC_DS_L1REG
                    // level 1 (every sure entry, most resolved ones) from a register: the row's chain
                    // keeps one LDS round trip (the tile's) instead of two
                    float lv = lv1;
                    if (__builtin_expect(__ballot(a != NONE && ((a >> 12) & 15u) != 1u) != 0ull, 0)) lv = lvl[(a >> 12) & 15u];
                    const float e = __uint_as_float(__float_as_uint(lv) | ((a & 0x800u) << 20)) * pn;
#else
                    const float e = value(a, pn);
#endif
                    if (a != NONE) {
                        const float t = W ? wi * e : e;
#if FLC_DS_LDSADD
                        // LDS fp32 add without return: one wave's LDS operations run in issue order, so
                        // each column still takes its rows' terms in row order; no read in the chain
                        if (!(t == 0.f)) atomicAdd(&tl[a & (HCHUNK - 1)], t);
#else
                        add(a & (HCHUNK - 1), t);
#endif
                    }
                }
            } else {
#pragma unroll 1
                for (int q = 0; q < 64; ++q) {
                    float pn, wi;
                    row_state(cur, q, pn, wi);
                    const uint32_t cnt = __builtin_amdgcn_readlane(cur.off, q) + __builtin_amdgcn_readlane(cur.cnt, q);
                    const uint32_t raw = dstg[wv][q >> 3][(q & 7) * 64 + lane];
                    const uint32_t a = (uint32_t)lane < cnt ? raw : NONE;
                    const float e = value(a, pn);
                    if (a != NONE) add(a & (HCHUNK - 1), W ? wi * e : e);
                    const int64_t row = i0 + q;
                    for (uint32_t kk = 64u + lane; kk < cnt; kk += 64) {
                        const uint32_t en = ws.ent16[(h * n + row) * DS_HCAP + kk];
                        const float ev = value(en, pn);
                        add(en & (HCHUNK - 1), W ? wi * ev : ev);
                    }
                }
                __builtin_amdgcn_s_waitcnt(0xC07F);                  // lgkmcnt(0): the slots are read
                nxt = ds_meta_raw(ws, h, n, rend, i0 + 64 + lane, w);
#pragma unroll
                for (int sl = 0; sl < 8; ++sl) dma(i0 + 64 + 8 * sl, sl);
            }
            cur = nxt;
        }
#else
        const uint16_t* hb = ws.ent16 + h * n * DS_HCAP + lane;
#pragma unroll
        for (int q = 0; q < AP; ++q) ra[q] = hb[min(r0 + q, n - 1) * DS_HCAP];
        // 64-row batches (the last one may be partial: its rows past the end have count 0) until
        // one holds a dense row; from there the rows go one at a time below
        for (; b < nb; ++b) {
            const int64_t i0 = r0 + b * 64;
            if (__ballot((cur.mode & DS_DENSE) != 0u) != 0ull) break;
            nxt = ds_meta(ws, h, n, rend, i0 + 64 + lane, w);
#pragma unroll 1
            for (int qb = 0; qb < 64; qb += AP) {
#pragma unroll
                for (int u = 0; u < AP; ++u) {
                    const int q = qb + u;
                    float pn, wi;
                    row_state(cur, q, pn, wi);
                    const uint32_t cnt = __builtin_amdgcn_readlane(cur.cnt, q);
                    const uint32_t a = (uint32_t)lane < cnt ? ra[u] : NONE;
                    const float e = value(a, pn);
                    if (a != NONE) add(a & (HCHUNK - 1), W ? wi * e : e);
                    if (__builtin_expect(cnt > 64u, 0)) {             // rare: the rest of a long list
                        const int64_t row = i0 + q;
                        for (uint32_t k = 64u + lane; k < cnt; k += 64) {
                            const uint32_t en = ws.ent16[(h * n + row) * DS_HCAP + k];
                            const float ev = value(en, pn);
                            add(en & (HCHUNK - 1), W ? wi * ev : ev);
                        }
                    }
                    ra[u] = hb[min(i0 + q + AP, n - 1) * DS_HCAP];
                }
            }
            cur = nxt;
        }
#endif
        // rows from the batch with a dense row on, one at a time (rare: a row outside its sample's
        // norm bounds, an overflowed item, a non-finite row or weight)
        for (int64_t row = r0 + b * 64; row < rend; ++row) {
            const uint32_t mode = ws.flags[row];
            const float pn = ws.pn[row], wi = W ? w[row] : 1.f;
            if (mode & DS_DENSE) {
                // dense row: every element of the half chunk, coalesced
                DsRow rr;
                rr.n = pn;
                rr.rn = ws.rpn[row];
                const uint32_t rk = ws.rk[row];
                rr.rk2 = rk ^ 0x27D4EB2Fu;
                rr.fast = (mode & DS_FAST) != 0u;
                const float* rp = rows.row(row) + hbase;
                for (int k = 0; k < HCHUNK / 64; ++k) {
                    const uint32_t e = (uint32_t)(k * 64 + lane);
                    if (e < (uint32_t)len) {
                        const uint32_t j = hbase + e;
                        const float ev = COMPAT ? ds_encode<true>(rp[e], j, 0u, us.u[row * us.uld + j], rr, tab, s, sf)
                                                : ds_encode<false>(rp[e], j, ds_hi8(j, rk), 0.0, rr, tab, s, sf);
                        add(e, W ? wi * ev : ev);
                    }
                }
            } else {
                const uint32_t cnt = ws.tabs[h * n + row].y + ws.cntr[h * n + row];
                for (uint32_t k = lane; k < cnt; k += 64) {
                    const uint32_t en = ws.ent16[(h * n + row) * DS_HCAP + k];
                    const float ev = value(en, pn);
                    add(en & (HCHUNK - 1), W ? wi * ev : ev);
                }
            }
        }
#else
#pragma unroll
        for (int q = 0; q < AP; ++q) fetch(cur, q, r0 + q, q);
        int64_t b = 0;
        for (; b < nb; ++b) {
            const int64_t i0 = r0 + b * 64;
            nxt = ds_meta(ws, h, n, rend, i0 + 64 + lane, w);
            // rows of this batch that need the general path: dense, or more than 64 entries here
            const uint64_t slow = __ballot((i0 + lane < rend) && ((cur.mode & DS_DENSE) || cur.cnt > 64u));
            if (slow == 0ull && i0 + 64 <= rend) {
                // straight line: per row its contribution, the add, the slot's refill
#pragma unroll 1
                for (int qb = 0; qb < 64; qb += AP) {
#pragma unroll
                    for (int u = 0; u < AP; ++u) {
                        const int q = qb + u;
                        float pn, wi;
                        row_state(cur, q, pn, wi);
                        const uint32_t a = ra[u];
                        const float e = value(a, pn);
                        if (a != NONE) add(a & (HCHUNK - 1), W ? wi * e : e);
                        refill(q, i0);
                    }
                }
            } else {
                const int nrow = (int)min((int64_t)64, rend - i0);
#pragma unroll 1
                for (int q = 0; q < 64; ++q) {
                    const int u = q % AP;
                    uint32_t a = NONE;
#pragma unroll
                    for (int z = 0; z < AP; ++z)
                        if (z == u) a = ra[z];
                    if (q < nrow) {
                        const int64_t row = i0 + q;
                        float pn, wi;
                        row_state(cur, q, pn, wi);
                        const uint32_t mode = __builtin_amdgcn_readlane(cur.mode, q);
                        if (mode & DS_DENSE) {
                            // dense row: every element of the half chunk, coalesced
                            DsRow rr;
                            rr.n = pn;
                            rr.rn = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(cur.rpn), q));
                            const uint32_t rk = __builtin_amdgcn_readlane(cur.rk, q);
                            rr.rk2 = rk ^ 0x27D4EB2Fu;
                            rr.fast = (mode & DS_FAST) != 0u;
                            const float* rp = rows.row(row) + hbase;
                            for (int k = 0; k < HCHUNK / 64; ++k) {
                                const uint32_t e = (uint32_t)(k * 64 + lane);
                                if (e < (uint32_t)len) {
                                    const uint32_t j = hbase + e;
                                    const float ev = COMPAT ? ds_encode<true>(rp[e], j, 0u, us.u[row * us.uld + j], rr, tab, s, sf)
                                                            : ds_encode<false>(rp[e], j, ds_hi8(j, rk), 0.0, rr, tab, s, sf);
                                    add(e, W ? wi * ev : ev);
                                }
                            }
                        } else {
                            if (a != NONE) {
                                const float e = value(a, pn);
                                add(a & (HCHUNK - 1), W ? wi * e : e);
                            }
                            const uint32_t cnt = __builtin_amdgcn_readlane(cur.cnt, q);
                            for (uint32_t e = 64u + lane; e < cnt; e += 64) {
                                const uint32_t en = ws.ent16[(h * n + row) * DS_HCAP + e];
                                const float ev = value(en, pn);
                                add(en & (HCHUNK - 1), W ? wi * ev : ev);
                            }
                        }
                    }
                    // refill the slot with row q + AP (dynamic slot: the loop is not unrolled)
                    const bool nb_ = q + AP >= 64;
                    const int qq = nb_ ? q + AP - 64 : q + AP;
                    const uint32_t cnt = __builtin_amdgcn_readlane(nb_ ? nxt.cnt : cur.cnt, qq);
                    const int64_t rown = i0 + q + AP;
                    const uint16_t* p = cnt ? ws.ent16 + (h * n + rown) * DS_HCAP : ws.ent16;
                    const uint32_t v = (uint32_t)lane < cnt ? (uint32_t)p[lane] : NONE;
#pragma unroll
                    for (int z = 0; z < AP; ++z)
                        if (z == u) ra[z] = v;
                }
            }
            cur = nxt;
        }
#endif
        if (!last) {
            for (int64_t i = lane; i < len; i += 64) part[hbase + i] = tl[i];
            continue;
        }
        // untouched columns: every contribution was +-0; the sequential fold gives -0 only if all
        // are -0.  Sign of row i's zero: C(x) = copysign(0, x) * norm (+0 for x == 0), times w_i.
        for (int k = 0; k < HCHUNK / 64; ++k) {
            const int e = k * 64 + lane;
            bool neg = e < len && __float_as_uint(tl[e]) == 0x80000000u;
            if (__ballot(neg) == 0ull) continue;
            const bool mine = neg;
            for (int64_t i = 0; i < n && __ballot(neg) != 0ull; ++i) {
                if (neg) {
                    const float xv = rows.row(i)[hbase + e];
                    const bool zs = (xv != 0.f) && (__float_as_uint(xv) >> 31);
                    const bool ws_ = W && (__float_as_uint(w[i]) >> 31);
                    neg = zs != ws_;
                }
            }
            if (mine) tl[e] = neg ? -0.f : 0.f;
        }
        for (int64_t i = lane; i < len; i += 64) out[hbase + i] = tl[i] / wt;
    }
}

// ------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------
// Filter grid.  The product build always takes the default; a -DFLC_TUNING build reads the
// A/B switches once per process (FLC_DS_GRID=res launches a resident-only grid; FLC_DS_GRIDPCT=p
// caps it at p % of the resident blocks when row groups run).
#ifndef FLC_DS_V2
#define FLC_DS_V2 0                  // device-RNG filter: classification pipelined into the next item (k_ds_filter2)
#endif
#ifndef FLC_DS_LDSPAD
#define FLC_DS_LDSPAD 5120           // row groups: extra LDS per filter block (bytes), room for the side tail
#endif
#ifndef FLC_DS_LASTPCT
#define FLC_DS_LASTPCT 100           // size of the last QSGD row group in % of the others (its tail is exposed)
#endif
static_assert(FLC_DS_LASTPCT >= 1 && FLC_DS_LASTPCT <= 100, "FLC_DS_LASTPCT: the last row group is 1..100 % of the others");
#ifndef FLC_DS_RG_SIDE
#define FLC_DS_RG_SIDE 1             // row groups: norm + resolve on the side stream too
#endif
#ifndef FLC_DS_RESGRID
#define FLC_DS_RESGRID 0             // k_ds_filter: a resident grid (one round of blocks, grid-stride items)
#endif
#ifndef FLC_DS_SIDE_FOLD_WG
#define FLC_DS_SIDE_FOLD_WG 0        // a non-last row group's fold (beside the next filter): grid cap, 0 = one per half
#endif
#ifndef FLC_DS_SIDE_RES_WG
#define FLC_DS_SIDE_RES_WG 0         // a non-last row group's resolve: grid cap, 0 = one wave per 64 items
#endif
#ifndef FLC_DS_PROBE_SIDE
#define FLC_DS_PROBE_SIDE 0          // A/B probes: 1 skip the side resolve, 2 the side fold, 3 both (outputs NOT valid)
#endif
#ifndef FLC_DS_PROBE_DEF
#define FLC_DS_PROBE_DEF 0           // A/B variant builds only (a probe's outputs are NOT valid)
#endif
struct DsVariant { bool resident; int gridpct; int probe; int64_t rb; int cring; };
static const DsVariant& ds_variant() {
    static const DsVariant v = [] {
        DsVariant r{false, 100, FLC_DS_PROBE_DEF, DS_RB, DS_RINGC};
        if (const char* e = tuning_env("FLC_DS_CRING")) r.cring = atoi(e);
        if (const char* e = tuning_env("FLC_DS_RB")) r.rb = std::max<int64_t>(1, atoll(e));
        if (const char* e = tuning_env("FLC_DS_PROBE")) r.probe = atoi(e);
        if (const char* e = tuning_env("FLC_DS_GRIDPCT")) r.gridpct = std::max(10, std::min(100, atoi(e)));
        if (const char* e = tuning_env("FLC_DS_GRID")) r.resident = !strcmp(e, "res");
        return r;
    }();
    return v;
}

static DsWs carve_ds(void* base, int64_t n, int64_t d, size_t* bytes) {
    Carver cv(base);
    const int64_t C = std::max<int64_t>(nchunks(d), 1), H = std::max<int64_t>(nhalves(d), 1);
    const int64_t nn = std::max<int64_t>(n, 1);
    DsWs w;
    w.G = (C + DS_FGS - 1) / DS_FGS;
    w.n = nn;
    w.cap = w.G * DS_GCAP;
    const size_t tabn = (size_t)std::max<int64_t>(H, w.G * DS_NH) * nn;         // + padding halves
    w.tabs = cv.take<uint2>(tabn);
    w.cntr = cv.take<uint32_t>(tabn);
    w.ent16 = cv.take<uint16_t>((size_t)nn * w.cap);
    w.enta = cv.take<uint2>((size_t)nn * w.cap);
    w.itm = cv.take<uint32_t>((size_t)nn * w.G);
    w.flags = cv.take<uint32_t>(nn);
    w.qc = cv.take<float>(nn);
    w.nlo = cv.take<float>(nn);
    w.nhi = cv.take<float>(nn);
    w.q0 = cv.take<float>(nn);
    w.q1 = cv.take<float>(nn);
    w.partial = cv.take<double>((size_t)nn * w.G);
    w.pn = cv.take<float>(nn);
    w.rpn = cv.take<float>(nn);
    w.rk = cv.take<uint32_t>(nn);
    w.part = cv.take<float>((size_t)std::max<int64_t>(d, 1));
    w.gtab = cv.take<float4>(DS_MAXS);
    if (bytes) *bytes = cv.bytes();
    return w;
}

// Path choice: the sparse path pays when the expected candidate share (s / sqrt(D), the hi8
// slack) keeps a filter item well inside its staging capacity.  The caller's hint
// (flc_codec_params.flags & FLC_PATH_MASK: FLC_PATH_SPARSE / FLC_PATH_DENSE) forces one; both
// paths give the same bits.

bool ds_eligible(const flc_codec_params* prm, const flc_pattern* pat, int64_t n, int64_t d) {
    if (prm->codec != FLC_STD_DITHERING || prm->norm != FLC_NORM_L2) return false;
    if (prm->s < 1 || prm->s > DS_MAXS - 1 || !prm->d_levels || n < 1 || d < 1) return false;
    if (d >= (int64_t)0x7FFFFFFF) return false;
    const int m = prm->flags & FLC_PATH_MASK;
    if (m) return m == FLC_PATH_SPARSE;
    const double share = 1.1 * (double)prm->s / sqrt((double)d) + 0.003;
    return share * DS_FGS * CHUNK <= (FLC_DS_V2 ? FLC_DS2_CAP : DS_GCAP) / 1.4;
}

size_t ds_workspace(const flc_codec_params* prm, int64_t n, int64_t d) {
    (void)prm;
    size_t b = 0;
    carve_ds(nullptr, n, d, &b);
    return b;
}

// Per-device side stream and events of the row-group pipeline (lazily created, mutex-guarded;
// enqueueing under the mutex keeps concurrent callers' event records and waits paired).
namespace {
struct DsCtx {
    hipStream_t side = nullptr;
    std::vector<hipEvent_t> ev;
};
std::mutex g_ds_mu;
std::map<int, DsCtx> g_ds_ctx;
}  // namespace

// Row groups whose norm + resolve overlap the next group's filter (one fold at the end): tuning
// builds FLC_DS_TAILOV=g, else 1
static int tail_groups(int64_t n) {
    static const int g = [] { const char* e = tuning_env("FLC_DS_TAILOV"); return e ? std::max(1, atoi(e)) : 1; }();
    return (int)std::max<int64_t>(1, std::min<int64_t>(g, n));
}

// Row groups of the pipeline: the caller's hint (FLC_ROW_GROUPS(g) in flags), else 2 for 128 rows
// or more.  Group g's norm, resolve and fold run on the side stream under group g + 1's filter,
// whose blocks reserve FLC_DS_LDSPAD bytes more LDS (5 instead of 6 per CU) so that the tail
// kernels find room beside them: C4 9.684 -> 9.554 ms per step, same allocation, two processes
// (round 4, profiles/r04); 3 groups ran 9.89 (one more filter launch boundary), and without the
// pad 2 groups ran 9.650 (round 3's version, the norm and resolve between the filters and no pad,
// was not faster than 1 group).
static int ds_groups(const flc_codec_params* prm, int64_t n) {
    const int g = (prm->flags >> 8) & 0xFF;
    return (int)std::max<int64_t>(1, std::min<int64_t>(g ? g : (n >= 128 ? 2 : 1), n));
}

int ds_run(const flc_codec_params* prm, const flc_pattern* pat, RowSrc rows, int64_t n, int64_t d, const float* w,
           float wt, float* pnorm_out, float* out, void* wsp, size_t ws_bytes, hipStream_t st) {
    const DsVariant& v = ds_variant();
    size_t need = 0;
    carve_ds(nullptr, n, d, &need);
    if (ws_bytes < need) { set_error("dithering (sparse): workspace %zu < %zu", ws_bytes, need); return FLC_ERR_WORKSPACE; }
    DsWs ws = carve_ds(wsp, n, d, nullptr);
    const int64_t client0 = pat ? pat->client0 : 0;
    const int64_t H = nhalves(d);
    const int K = ds_groups(prm, n);
    // compat: the caller's float64 uniforms (the reference's numpy stream) instead of device draws
    const bool compat = pat && pat->d_uniforms;
    const UniformSrc us{compat ? pat->d_uniforms : nullptr, (pat && pat->uniforms_ld) ? pat->uniforms_ld : d};

    hipEvent_t filt_ev = nullptr;
    auto filter = [&](int64_t r0, int64_t rn, hipStream_t s2 = nullptr, bool beside = false) -> int {
        // s2: the row group's norm / resolve go to this stream (after an event on st), under the
        // next group's filter
        auto kern = compat ? (v.cring == 8 ? k_ds_filter<8, DS_GCAP, 0, true> : k_ds_filter<DS_RINGC, DS_GCAP, 0, true>)
                  : v.probe == 1 ? k_ds_filter<16, DS_GCAP, 1> : v.probe == 2 ? k_ds_filter<16, DS_GCAP, 2>
                  : v.probe == 3 ? k_ds_filter<16, DS_GCAP, 3> : v.probe == 4 ? k_ds_filter<16, DS_GCAP, 4>
                  : v.probe == 5 ? k_ds_filter<16, DS_GCAP, 5> : v.probe == 6 ? k_ds_filter<16, DS_GCAP, 6>
                  : FLC_DS_V2 ? k_ds_filter2<16, FLC_DS2_CAP> : k_ds_filter<16, DS_GCAP>;
        int gw = (int)std::max<int64_t>(1, std::min<int64_t>((rn * ws.G + 3) / 4, 32768));
        // row groups (s2: the group's tail runs beside the next group's filter): the filter's
        // blocks reserve FLC_DS_LDSPAD more bytes of LDS, so one block fewer fits a CU and the
        // side stream's tail kernels find room without waiting for a filter block to retire
        const size_t pad = s2 ? (size_t)FLC_DS_LDSPAD : 0u;
        if (FLC_DS_RESGRID || v.resident || (K > 1 && v.gridpct < 100)) {
            // resident grid: exactly the blocks that fit the chip at once (the LDS pad counted),
            // each walking its items grid-stride, so no block retires before the end — no partial
            // last round of blocks, and the side stream's kernels get only the room left beside
            // the filter instead of every slot a retiring filter block frees
            int per = 0, dev = 0, cus = 0;
            if (hipGetDevice(&dev) == hipSuccess &&
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
                hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, 256, pad) == hipSuccess && per > 0)
                gw = std::min(gw, std::max(1, per * cus * (K > 1 ? v.gridpct : 100) / 100));
        }
        { ProfScope _ps("k_ds_filter", st);
        hipLaunchKernelGGL(kern, dim3(gw), dim3(256), pad, st, rows, n, r0, rn, std::min<int64_t>(v.rb, rn), d, ws, us); }
        FLC_CHECK_LAUNCH("k_ds_filter");
        hipStream_t sr = st;
        if (s2) {
            FLC_CHECK_HIP(hipEventRecord(filt_ev, st));
            FLC_CHECK_HIP(hipStreamWaitEvent(s2, filt_ev, 0));
            sr = s2;
        }
        hipLaunchKernelGGL(k_ds_final, dim3((unsigned)((rn + 3) / 4)), dim3(256), 0, sr, r0, rn, ws, w, pnorm_out);
        FLC_CHECK_LAUNCH("k_ds_final");
        int rb = (int)std::max<int64_t>(1, std::min<int64_t>(((rn + 63) / 64 * ws.G + 3) / 4, 8192));
        // beside the next group's filter: a bounded grid (grid-stride), so the side kernel holds a
        // fixed share of the CUs instead of taking every slot a retiring filter block frees
        if (beside && FLC_DS_SIDE_RES_WG > 0) rb = std::min(rb, FLC_DS_SIDE_RES_WG);
        if (!(beside && (FLC_DS_PROBE_SIDE & 1)))             // probe builds only (outputs NOT valid)
        { ProfScope _ps("k_ds_resolve", sr);
        hipLaunchKernelGGL(compat ? k_ds_resolve<true> : k_ds_resolve<false>, dim3(rb), dim3(256), 0, sr, n, r0, rn, ws,
                           prm->d_levels, prm->s, us); }
        FLC_CHECK_LAUNCH("k_ds_resolve");
        return FLC_OK;
    };
    auto accum = [&](int64_t r0, int64_t rn, int first, int last, hipStream_t s2, bool beside = false) -> int {
        int ab = (int)std::max<int64_t>(1, std::min<int64_t>((H + DS_AW - 1) / DS_AW, 32768));
        if (beside && FLC_DS_SIDE_FOLD_WG > 0) ab = std::min(ab, FLC_DS_SIDE_FOLD_WG);
        ProfScope _ps("k_ds_accum", s2);
        auto kern = w ? (compat ? k_ds_accum<true, DS_AP, true> : k_ds_accum<true, DS_AP, false>)
                      : (compat ? k_ds_accum<false, DS_AP, true> : k_ds_accum<false, DS_AP, false>);
        hipLaunchKernelGGL(kern, dim3(ab), dim3(64 * DS_AW), 0, s2, rows, n, r0, rn, first, last, d, ws, prm->d_levels, prm->s, w,
                           wt, ws.part, out, us);
        FLC_CHECK_LAUNCH("k_ds_accum");
        return FLC_OK;
    };

    auto sample = [&](int64_t a, int64_t b, hipStream_t sx) -> int {
        if (b <= a) return FLC_OK;
        ProfScope _ps("k_ds_sample", sx);
        hipLaunchKernelGGL(k_ds_sample, dim3((unsigned)(b - a)), dim3(DS_SNT), 0, sx, rows, n, d, prm->d_levels, prm->s, prm->seed,
                           client0, ws, a);
        FLC_CHECK_LAUNCH("k_ds_sample");
        return FLC_OK;
    };
    const int TO = tail_groups(n);
    // row groups (K >= 2): only group 0's sample before its filter; the other rows' samples run on
    // the side stream beside it and group 1's filter waits for them
    const bool split = FLC_DS_SPLIT_SAMPLE && K >= 2;
    if (!split)
        if (int rc = sample(0, n, st)) return rc;
    if (K == 1 && TO <= 1) {
        int rc = filter(0, n);
        if (rc) return rc;
        return accum(0, n, 1, 1, st);
    }
    // Row-group pipeline: the fold of group g (side stream, latency-bound) runs under the filter
    // of group g + 1 (caller stream, HBM-bound); the groups' folds continue one another's tiles
    // through `part`, in row order.
    int dev = 0;
    FLC_CHECK_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_ds_mu);
    DsCtx& cx = g_ds_ctx[dev];
    if (!cx.side) {
        // the fold is latency-bound and short: it gets the dispatcher's priority over the filter
        int lo = 0, hi = 0;
        FLC_CHECK_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
        FLC_CHECK_HIP(hipStreamCreateWithPriority(&cx.side, hipStreamNonBlocking, hi));
    }
    while ((int)cx.ev.size() < std::max(K, TO) + 4) {
        hipEvent_t e;
        FLC_CHECK_HIP(hipEventCreateWithFlags(&e, FLC_SYNC_EVENT_FLAGS));
        cx.ev.push_back(e);
    }
    if (K == 1) {
        // Tail overlap: row group g's norm and resolve (latency-bound, little memory traffic) run on
        // the side stream under the filter of group g + 1; one fold of all rows at the end.
        // (A stream's events are reused in order: a record after the wait that consumed it.)
        for (int g = 0; g < TO; ++g) {
            const int64_t r0 = n * g / TO, r1 = n * (g + 1) / TO;
            filt_ev = cx.ev[g];
            int rc = filter(r0, r1 - r0, cx.side);
            if (rc) return rc;
        }
        FLC_CHECK_HIP(hipEventRecord(cx.ev[TO], cx.side));
        FLC_CHECK_HIP(hipStreamWaitEvent(st, cx.ev[TO], 0));
        return accum(0, n, 1, 1, st);
    }
    const int EV_S0 = std::max(K, TO) + 2, EV_S1 = EV_S0 + 1;
    if (split) {
        const int64_t rs1 = group_row(n, K, 1, FLC_DS_LASTPCT);
        FLC_CHECK_HIP(hipEventRecord(cx.ev[EV_S0], st));                   // after the work queued before
        FLC_CHECK_HIP(hipStreamWaitEvent(cx.side, cx.ev[EV_S0], 0));
        if (int rc = sample(0, rs1, st)) return rc;
        if (int rc = sample(rs1, n, cx.side)) return rc;
        FLC_CHECK_HIP(hipEventRecord(cx.ev[EV_S1], cx.side));
    }
    for (int g = 0; g < K; ++g) {
        const int64_t r0 = group_row(n, K, g, FLC_DS_LASTPCT), r1 = group_row(n, K, g + 1, FLC_DS_LASTPCT);
        if (split && g == 1) FLC_CHECK_HIP(hipStreamWaitEvent(st, cx.ev[EV_S1], 0));
        int rc;
        if (FLC_DS_RG_SIDE) {
            // the group's whole tail (norm, resolve, fold) on the side stream, under the next
            // group's filter
            filt_ev = cx.ev[g];
            rc = filter(r0, r1 - r0, cx.side, g < K - 1);
        } else {
            rc = filter(r0, r1 - r0);
            if (!rc) {
                FLC_CHECK_HIP(hipEventRecord(cx.ev[g], st));
                FLC_CHECK_HIP(hipStreamWaitEvent(cx.side, cx.ev[g], 0));
            }
        }
        if (rc) return rc;
        if (!(g < K - 1 && (FLC_DS_PROBE_SIDE & 2)))         // probe builds only (outputs NOT valid)
            rc = accum(r0, r1 - r0, g == 0, g == K - 1, cx.side, g < K - 1);
        if (rc) return rc;
    }
    FLC_CHECK_HIP(hipEventRecord(cx.ev[K], cx.side));
    FLC_CHECK_HIP(hipStreamWaitEvent(st, cx.ev[K], 0));
    return FLC_OK;
}

}  // namespace flc
