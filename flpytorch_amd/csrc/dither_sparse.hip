// Sparse fused standard dithering / QSGD encode + reduce: device-RNG mode, p = 2 norm.
// fl_pytorch/utils/compressors.py:270-299 (the codec; qsgd = std dithering with p = 2, 95-101) and
// the serverGradient fold (algorithms.py:1748-1770), reading every client row from HBM ONCE.
//
// Why a sparse path: the encode needs the row's norm before any element, so the dense path reads
// every row twice (norm pass + encode pass, codecs.hip).  But QSGD's output is sparse: element j
// is nonzero only if y_j = |x_j| / ||x||_2 >= l1 (the first level, 1/s) or its draw goes up, so
//     E[nonzeros] <= sum_j min(1, y_j / l1) <= ||x||_1 / (l1 ||x||_2) <= s sqrt(D)
// for ANY row (2.5 % of the elements at s = 127, D = 25 M).  One streaming pass can therefore
// accumulate the norm AND keep every element that could be nonzero, using a LOWER bound n_lo of
// the norm (a spread sample's estimate, discounted): the candidates are then encoded exactly, with
// the exact norm, by the chunk owners of the fold.
//
//   sample  : per row, sum of squares of a spread 16 K-element sample -> n_lo, the candidate scale
//             qc = 256 (1 + 2^-18) / (l1 n_lo), the device-RNG row key.
//   filter  : ONE pass over every row: float64 sum of squares per 8192-element item (fixed slots),
//             and every element passing  fma(|x|, qc, hi8) > 254.98  appended (idx, x) to the
//             row's candidate list, per 4096-element chunk (tab[c][row]).  hi8 is the top byte of
//             the element's draw (common.hpp: one group hash per 4 elements), so the test costs a
//             quarter hash per element.
//   final   : per row, norm = RN(sqrt(sum of the partials in a fixed order)); the row is folded
//             DENSE (every element re-read and encoded) if the norm is below n_lo (sample
//             misjudged), not finite, its weight not finite, or its list overflowed.
//   accum   : one wave owns a 4096-element chunk as an fp32 LDS tile and folds the rows in order:
//             each candidate is encoded exactly (DitherOp, the dense path's functor) and nonzero
//             contributions are added; untouched columns get the sign of zero the sequential fold
//             of the all-zero contributions gives (-0 only if every row contributes -0).
//
// The candidate test is conservative (never drops a nonzero).  For n >= n_lo, in the first level
// interval [0, l1] the encode keeps l0 = 0 iff  h < ceil(p 2^32),  p = RN(RN(y - l1) / (-l1)),
// y = RN(|x| / n), and  p >= 1 - y / l1 - 2^-23,  y <= (|x| / n_lo)(1 + 2^-24).  A nonzero output
// has h >= p 2^32, so hi8 = h >> 24 > 256 p - 1 >= 255 - 256 |x| (1 + 2^-24) / (l1 n_lo) - 2^-15,
// and  |x| qc + hi8 > 255 - 2^-15;  the fp32 fma loses < 2^-14 there, so  > 254.98  keeps every
// nonzero.  Elements in higher intervals (y >= l1) have |x| qc >= 256.
#include "chunks.hpp"
#include "codec_ops.hpp"

namespace flc {

constexpr uint32_t DS_DENSE = 1u, DS_OVER = 2u;
constexpr int DS_FGS = 2;                  // chunks per filter work item (8192 elements)
constexpr int DS_GCAP = 512;               // staged candidates per item (6.25 %; more -> row overflow)
constexpr int DS_SMAX = 16384;             // sample elements per row
constexpr uint32_t DS_SENT = 0x7FBADBADu;  // LDS tile: untouched column (a signalling NaN: never computed)
constexpr float DS_QT = 254.98f;
constexpr int DS_MAXS = 512;               // level table entries kept in LDS by the fold
static_assert(DS_GCAP % 64 == 0, "copy-out runs in whole wave slots");

struct DsWs {
    uint2* tab;           // [C][N] (offset, count) of each row's candidates in chunk c
    uint32_t* ent_idx;    // [N][cap] element index within the row
    float* ent_val;       // [N][cap] x
    uint32_t* rowcnt;     // [N * RCS] entries used
    uint32_t* flags;      // [N] DS_*
    float* qc;            // [N] candidate scale
    float* nlo;           // [N] norm lower bound the scale assumes
    double* partial;      // [N][G] per-item sums of squares
    float* pn;            // [N] norm
    uint32_t* rk;         // [N] device-RNG row key
    int64_t cap;
    int64_t G;            // filter items per row
};

// ------------------------------------------------------------------------------------------
// Sample: one workgroup per row.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_ds_sample(RowSrc rows, int64_t n, int64_t d, const float* __restrict__ levels,
                                                   uint64_t seed, int64_t client0, DsWs ws) {
    __shared__ double r2[4], r4[4];
    const int64_t row = blockIdx.x;
    if (row >= n) return;
    const float* r = rows.row(row);
    double a2 = 0.0, a4 = 0.0;
    int64_t S;
    if (d <= DS_SMAX) {
        S = d;
        for (int64_t i = threadIdx.x; i < d; i += 256) {
            const double v = (double)r[i] * (double)r[i];
            a2 += v;
            a4 += v * v;
        }
    } else {
        // 64 pieces of 256 contiguous elements spread evenly; thread t reads element t of 8 pieces
        // per round trip
        constexpr int P = DS_SMAX / 256;
        S = DS_SMAX;
        for (int p0 = 0; p0 < P; p0 += 8) {
            float x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) x[u] = r[((int64_t)(p0 + u) * (d - 256)) / (P - 1) + threadIdx.x];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
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
        a2 = (r2[0] + r2[1]) + (r2[2] + r2[3]);
        a4 = (r4[0] + r4[1]) + (r4[2] + r4[3]);
        const float l0 = levels[0], l1 = levels[1];
        const bool bad = !(l0 == 0.f) || !(l1 > 0.f);   // the bound needs levels 0 < l1 < ...
        double nlo;
        if (S == d) {
            nlo = sqrt(a2) * (1.0 - 0x1p-20);              // the whole row: the norm itself
        } else {
            // estimate of the sum of squares, discounted by 6 sigma of the sample mean + 2 %
            const double m = (double)S, mean2 = a2 / m;
            const double var = fmax(a4 / m - mean2 * mean2, 0.0);
            const double rel = sqrt(var / m) / mean2;      // NaN/inf when mean2 == 0 or overflow
            const double f = fmin(fmax(1.0 - 6.0 * rel - 0.02, 0.25), 0.97);
            nlo = sqrt(f * mean2 * (double)d);
        }
        float nlof = (float)nlo;
        if (!(nlof >= 0.f) || !(nlof <= 3.0e38f)) nlof = 0.f;
        const double qcd = 256.0 * (1.0 + 0x1p-18) / ((double)l1 * (double)nlof);   // +inf for nlof 0
        float qc = (float)(qcd * (1.0 + 0x1p-22));         // rounded up past the conversion
        if (!(qc >= 0.f)) qc = __builtin_huge_valf();
        if (bad) qc = 0.f;                                 // row is folded dense anyway
        ws.qc[row] = qc;
        ws.nlo[row] = nlof;
        ws.flags[row] = bad ? DS_DENSE : 0u;
        ws.rowcnt[row * RCS] = 0;
        ws.rk[row] = rowkey(client_key(seed, client0 + row));
    }
}

// ------------------------------------------------------------------------------------------
// Filter: the TopK fast filter's structure (select.hip k_topk_filter_fast: RING-deep buffer-load
// pipeline across chunks and items, wave-private double-buffered LDS staging, one reservation
// atomic per item consumed an item later) with the dithering candidate test and the norm.
// ------------------------------------------------------------------------------------------
template <int RING>
__global__ __launch_bounds__(256) void k_ds_filter(RowSrc rows, int64_t n, int64_t d, DsWs ws) {
    constexpr int FGS = DS_FGS;
    static_assert(16 % RING == 0, "ring must divide the 16 loads of a chunk");
    __shared__ uint32_t st_idx[2][4][DS_GCAP];
    __shared__ float st_val[2][4][DS_GCAP];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t C = nchunks(d);
    const int64_t G = ws.G;
    const int64_t items = n * G;
    const int64_t stride = (int64_t)gridDim.x * 4;
    int64_t it = (int64_t)blockIdx.x * 4 + wv;
    if (it >= items) return;
    const uint32_t lphi = (uint32_t)lane * 0x9E3779B1u;    // group index g = c*1024 + 64 L + lane
    float4 ring[RING];
    int64_t row = it / G;
    int64_t c = (it - row * G) * FGS;
    auto rs = chunk_rsrc(rows.row_s(row), c * CHUNK, d);
#pragma unroll
    for (int L = 0; L < RING - 1; ++L) {
        ring[L] = load_q(rs, lane, L);
        __builtin_amdgcn_sched_barrier(0);
    }
    bool pv = false;
    int64_t prow = 0, pc0 = 0;
    uint64_t pcc = 0;
    uint32_t ptot = 0, pres = 0;
    int par = 0;
    auto finish = [&](int pb) {
        uint32_t base = 0;
        bool fits = ptot <= DS_GCAP;
        if (fits && ptot) {
            base = __shfl(pres, 0, WAVE);
            fits = (int64_t)base + ptot <= ws.cap;
        }
        if (lane < FGS && pc0 + lane < C) {
            uint32_t off = 0, cc = 0;
#pragma unroll
            for (int u = 0; u < FGS; ++u) {
                const uint32_t cu = (uint32_t)(pcc >> (16 * u)) & 0xFFFFu;
                off += u < lane ? cu : 0u;
                cc = u == lane ? cu : cc;
            }
            ws.tab[(pc0 + lane) * n + prow] = make_uint2(base + off, fits ? cc : 0u);
        }
        if (!fits && lane == 0) atomicOr(&ws.flags[prow], DS_OVER);
        if (fits) {
            const uint32_t* si = st_idx[pb][wv];
            const float* sv = st_val[pb][wv];
            uint32_t* oi = ws.ent_idx + prow * ws.cap + base;
            float* ov = ws.ent_val + prow * ws.cap + base;
#pragma unroll
            for (int k = 0; k < DS_GCAP / 64; ++k) {
                const uint32_t e = (uint32_t)(k * 64 + lane);
                if (e < ptot) { oi[e] = si[e]; ov[e] = sv[e]; }
            }
        }
    };
    while (it < items) {
        const float qc = sload(ws.qc + row);
        const uint32_t rk = sload(ws.rk + row);
        const int64_t gi = it - row * G;
        const int64_t nit = it + stride;
        uint32_t* si = st_idx[par][wv];
        float* sv = st_val[par][wv];
        uint32_t cnt = 0;
        uint64_t ccp = 0;
        double a2 = 0.0;
        const int64_t cg0 = c;
        int64_t nrow = row, nc = c;
#pragma unroll
        for (int sub = 0; sub < FGS; ++sub, ++c) {
            const int64_t j0 = c * CHUNK;
            __amdgpu_buffer_rsrc_t rsn;
            if (sub + 1 < FGS) {
                rsn = chunk_rsrc(rows.row_s(row), j0 + CHUNK, d);
            } else if (nit < items) {
                nrow = nit / G;
                nc = (nit - nrow * G) * FGS;
                rsn = chunk_rsrc(rows.row_s(nrow), nc * CHUNK, d);
            } else {
                rsn = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(rows.row_s(row)), (short)0, 0, 0x00020000);
            }
            const uint32_t cnt0 = cnt;
            // element index of (L, q): jb + 256 L + q (opaque: keeps the 64 constants out of VGPRs)
            uint32_t jb = (uint32_t)j0 + (uint32_t)lane * 4u;
            asm volatile("" : "+v"(jb));
            const uint32_t gb = lphi + (uint32_t)(c * 1024) * 0x9E3779B1u + rk;   // hash input of L = 0
#pragma unroll
            for (int L = 0; L < 16; ++L) {
                const int P = L + RING - 1;
                ring[P % RING] = P < 16 ? load_q(rs, lane, P) : load_q(rsn, lane, P - 16);
                const float4 x = ring[L % RING];
                const uint32_t hg = fmix32(gb + (uint32_t)(L * 64) * 0x9E3779B1u);
                const float vq[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    a2 = fma((double)vq[q], (double)vq[q], a2);
                    const float hi = (float)((hg >> (8 * q)) & 0xFFu);
                    // no range test: past the row end the loads return 0, and a zero candidate
                    // encodes to 0 (never folded); NaN from 0 * inf (qc = inf) is not a candidate
                    const bool f = fmaf(fabsf(vq[q]), qc, hi) > DS_QT;
                    const uint64_t m = __ballot(f);
                    // branch-free compaction: position = cnt + candidates in lower lanes; an item
                    // past DS_GCAP overflows (its row is folded dense), so wrapping is harmless
                    const uint32_t pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                             __builtin_amdgcn_mbcnt_lo((uint32_t)m, cnt)) & (DS_GCAP - 1);
                    if (f) { si[pos] = jb + (uint32_t)(L * 256 + q); sv[pos] = vq[q]; }
                    cnt += (uint32_t)__popcll(m);
                }
                // keep the norm's fma chain here: left alone, the compiler sinks all 128 of an
                // item's fmas to its end and holds the 128 x values live (218 VGPRs)
                asm volatile("" : "+v"(a2));
            }
            ccp |= (uint64_t)min(cnt - cnt0, 0xFFFFu) << (16 * (c - cg0));
            rs = rsn;
        }
        a2 = wave_sum(a2);                                   // fixed butterfly: deterministic
        if (lane == 0) ws.partial[row * G + gi] = a2;
        if (pv) finish(par ^ 1);
        uint32_t res = 0;
        if (cnt && cnt <= DS_GCAP && lane == 0) res = atomicAdd(&ws.rowcnt[row * RCS], cnt);
        pv = true; prow = row; pc0 = cg0; pcc = ccp; ptot = cnt; pres = res;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        par ^= 1;
        it = nit;
        row = nrow;
        c = nc;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    finish(par ^ 1);
}

// ------------------------------------------------------------------------------------------
// Norm and row mode: one wave per row.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_ds_final(int64_t n, DsWs ws, const float* __restrict__ w,
                                                  float* __restrict__ pnorm_out) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n) return;
    double a = 0.0;
    for (int64_t k = lane; k < ws.G; k += 64) a += ws.partial[row * ws.G + k];
    a = wave_sum(a);
    if (lane == 0) {
        const float nv = (float)sqrt(a);
        ws.pn[row] = nv;
        if (pnorm_out) pnorm_out[row] = nv;
        uint32_t fl = ws.flags[row];
        const bool wbad = w && !(fabsf(w[row]) <= 3.4028235e38f);
        if (!(nv >= ws.nlo[row]) || !(nv <= 3.4028235e38f) || (fl & DS_OVER) || wbad) fl |= DS_DENSE;
        ws.flags[row] = fl;
    }
}

// ------------------------------------------------------------------------------------------
// Chunk-owner fold.  One wave per chunk, fp32 LDS tile, rows in order; per row the candidate list
// (first 128 entries from a ring of AP rows in flight, the rest read in place) or, for DENSE rows,
// the chunk of x itself.  Contributions are W ? w_i * C(x)_j : C(x)_j with C the exact encode.
// ------------------------------------------------------------------------------------------
constexpr int DS_AP = 8;

struct DsMeta {
    uint2 te;
    float pn, w;
    uint32_t rk, mode;
};

__device__ inline DsMeta ds_meta(const DsWs& ws, int64_t c, int64_t n, int64_t r, const float* w) {
    DsMeta m;
    m.te = make_uint2(0, 0);
    m.pn = 1.f; m.w = 1.f; m.rk = 0; m.mode = 0;
    if (r < n) {
        m.te = ws.tab[c * n + r];
        m.pn = ws.pn[r];
        m.rk = ws.rk[r];
        m.mode = ws.flags[r] & DS_DENSE;
        if (w) m.w = w[r];
    }
    return m;
}

template <bool W>
__global__ __launch_bounds__(256) void k_ds_accum(RowSrc rows, int64_t n, int64_t d, DsWs ws,
                                                  const float* __restrict__ levels, int s,
                                                  const float* __restrict__ w, float wt, float* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) float tile[4][CHUNK];
    __shared__ __attribute__((aligned(16))) float4 tab[DS_MAXS];
    const bool tab_ok = load_table(levels, s, tab);
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t C = nchunks(d);
    float* tl = tile[wv];
    const int64_t nb = (n + 63) / 64;
    DitherOp<false, false> op;
    op.us = UniformSrc{nullptr, 0};
    op.rt = RowTabs{nullptr, nullptr, nullptr, nullptr};
    op.s = s;
    op.sf = (float)s;
    op.urow = nullptr;
    op.fast = false;
    op.tab_ok = tab_ok;
    for (int64_t c = (int64_t)blockIdx.x * 4 + wv; c < C; c += (int64_t)gridDim.x * 4) {
        for (int i = lane; i < CHUNK; i += 64) tl[i] = __uint_as_float(DS_SENT);
        const uint32_t cbase = (uint32_t)(c * CHUNK);
        const int64_t len = min((int64_t)CHUNK, d - (int64_t)cbase);
        DsMeta cur = ds_meta(ws, c, n, lane, w), nxt;
        uint32_t ri[DS_AP][2];
        float rv[DS_AP][2];
        auto fetch = [&](const DsMeta& m, int q, int64_t row, int slot) {
            const uint32_t off = __builtin_amdgcn_readlane(m.te.x, q), cnt = __builtin_amdgcn_readlane(m.te.y, q);
            const auto di = list_rsrc(ws.ent_idx + row * ws.cap + off, cnt);
            const auto dv = list_rsrc(ws.ent_val + row * ws.cap + off, cnt);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t e = (uint32_t)lane + 64u * h;
                const uint32_t x = __builtin_amdgcn_raw_buffer_load_b32(di, lane * 4, h * 256, 0);
                ri[slot][h] = e < cnt ? x : 0xFFFFFFFFu;
                rv[slot][h] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(dv, lane * 4, h * 256, 0));
            }
        };
        auto fold = [&](uint32_t ix, float xv, float wi) {
            const uint32_t loc = ix - cbase;
            if (loc < (uint32_t)CHUNK) {
                const float e = op.template apply<false>(xv, (int64_t)ix, colbase(ix), tab);
                const float t = W ? wi * e : e;
                if (!(t == 0.f)) {
                    const float o = tl[loc];
                    tl[loc] = (__float_as_uint(o) == DS_SENT) ? t : o + t;
                }
            }
        };
#pragma unroll
        for (int q = 0; q < DS_AP; ++q) fetch(cur, q, q, q);
        for (int64_t b = 0; b < nb; ++b) {
            const int64_t i0 = b * 64;
            nxt = ds_meta(ws, c, n, i0 + 64 + lane, w);
            for (int qb = 0; qb < 64; qb += DS_AP) {
#pragma unroll
                for (int u = 0; u < DS_AP; ++u) {
                    const int q = qb + u;
                    const int64_t row = i0 + q;
                    if (row < n) {
                        op.dn = make_div(__uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(cur.pn), q)));
                        op.rk = __builtin_amdgcn_readlane(cur.rk, q);
                        const float wi = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(cur.w), q));
                        const uint32_t mode = __builtin_amdgcn_readlane(cur.mode, q);
                        if (mode) {
                            // dense row: every element of the chunk, coalesced
                            const float* rp = rows.row(row) + cbase;
                            for (int k = 0; k < CHUNK / 64; ++k) {
                                const int e = k * 64 + lane;
                                if (e < len) fold(cbase + (uint32_t)e, rp[e], wi);
                            }
                        } else {
                            fold(ri[u][0], rv[u][0], wi);
                            fold(ri[u][1], rv[u][1], wi);
                            const uint32_t cnt = __builtin_amdgcn_readlane(cur.te.y, q);
                            if (cnt > 128u) {
                                const uint32_t off = __builtin_amdgcn_readlane(cur.te.x, q);
                                for (uint32_t e = 128u + lane; e < cnt; e += 64)
                                    fold(ws.ent_idx[row * ws.cap + off + e], ws.ent_val[row * ws.cap + off + e], wi);
                            }
                        }
                    }
                    // refill the slot with row q + AP (next batch's meta past the batch end)
                    if (q + DS_AP < 64) fetch(cur, q + DS_AP, row + DS_AP, u);
                    else fetch(nxt, q + DS_AP - 64, row + DS_AP, u);
                }
            }
            cur = nxt;
        }
        // untouched columns: every contribution was +-0; the sequential fold gives -0 only if all
        // are -0.  Sign of row i's zero: C(x) = copysign(0, x) * norm (+0 for x == 0), times w_i.
        for (int k = 0; k < CHUNK / 64; ++k) {
            const int e = k * 64 + lane;
            bool neg = e < len && __float_as_uint(tl[e]) == DS_SENT;
            if (__ballot(neg) == 0ull) continue;
            const bool mine = neg;
            for (int64_t i = 0; i < n && __ballot(neg) != 0ull; ++i) {
                if (neg) {
                    const float xv = rows.row(i)[cbase + e];
                    const bool zs = (xv != 0.f) && (__float_as_uint(xv) >> 31);
                    const bool ws_ = W && (__float_as_uint(w[i]) >> 31);
                    neg = zs != ws_;
                }
            }
            if (mine) tl[e] = neg ? -0.f : 0.f;
        }
        for (int64_t i = lane; i < len; i += 64) out[cbase + i] = tl[i] / wt;
    }
}

// ------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------
static int64_t ds_cap(int s, int64_t d) {
    // 2x the s sqrt(D) bound on the expected nonzeros (n_lo >= n / 2), the hi8 slack and margin
    const double b = 2.0 * (double)s * sqrt((double)d) + (double)d / 256.0 + 2.0 * DS_FGS * CHUNK;
    int64_t cap = std::min<int64_t>(d, (int64_t)b);
    return std::max<int64_t>((cap + 3) & ~int64_t(3), 4);
}

static DsWs carve_ds(void* base, int s, int64_t n, int64_t d, size_t* bytes) {
    Carver cv(base);
    const int64_t C = std::max<int64_t>(nchunks(d), 1), nn = std::max<int64_t>(n, 1);
    DsWs w;
    w.cap = ds_cap(s, d);
    w.G = (C + DS_FGS - 1) / DS_FGS;
    w.tab = cv.take<uint2>((size_t)C * nn);
    w.ent_idx = cv.take<uint32_t>((size_t)nn * w.cap);
    w.ent_val = cv.take<float>((size_t)nn * w.cap);
    w.rowcnt = cv.take<uint32_t>((size_t)nn * RCS);
    w.flags = cv.take<uint32_t>(nn);
    w.qc = cv.take<float>(nn);
    w.nlo = cv.take<float>(nn);
    w.partial = cv.take<double>((size_t)nn * w.G);
    w.pn = cv.take<float>(nn);
    w.rk = cv.take<uint32_t>(nn);
    if (bytes) *bytes = cv.bytes();
    return w;
}

// Path choice: the sparse path pays when the expected candidate share (s / sqrt(D), the hi8
// slack) keeps a filter item well inside its staging capacity.  FLC_DITHER_PATH=sparse|dense
// forces one (tests, tuning).
int ds_mode_env() {
    const char* e = getenv("FLC_DITHER_PATH");
    if (!e) return 0;
    if (!strcmp(e, "sparse")) return 1;
    if (!strcmp(e, "dense")) return 2;
    return 0;
}

bool ds_eligible(const flc_codec_params* prm, const flc_pattern* pat, int64_t n, int64_t d) {
    if (prm->codec != FLC_STD_DITHERING || prm->norm != FLC_NORM_L2) return false;
    if (pat && pat->d_uniforms) return false;                    // compat draws: dense path
    if (prm->s < 1 || prm->s > DS_MAXS - 1 || !prm->d_levels || n < 1 || d < 1) return false;
    if (d >= (int64_t)0x7FFFFFFF) return false;
    const int m = ds_mode_env();
    if (m) return m == 1;
    const double share = 1.1 * (double)prm->s / sqrt((double)d) + 0.003;
    return share * DS_FGS * CHUNK <= DS_GCAP / 1.4;
}

size_t ds_workspace(const flc_codec_params* prm, int64_t n, int64_t d) {
    size_t b = 0;
    carve_ds(nullptr, prm->s, n, d, &b);
    return b;
}

int ds_run(const flc_codec_params* prm, const flc_pattern* pat, RowSrc rows, int64_t n, int64_t d, const float* w,
           float wt, float* pnorm_out, float* out, void* wsp, size_t ws_bytes, hipStream_t st) {
    size_t need = 0;
    carve_ds(nullptr, prm->s, n, d, &need);
    if (ws_bytes < need) { set_error("dithering (sparse): workspace %zu < %zu", ws_bytes, need); return FLC_ERR_WORKSPACE; }
    DsWs ws = carve_ds(wsp, prm->s, n, d, nullptr);
    const int64_t client0 = pat ? pat->client0 : 0;
    const int64_t C = nchunks(d);
    { ProfScope _ps("k_ds_sample", st);
    hipLaunchKernelGGL(k_ds_sample, dim3((unsigned)n), dim3(256), 0, st, rows, n, d, prm->d_levels, prm->seed, client0, ws); }
    FLC_CHECK_LAUNCH("k_ds_sample");
    {
        const int64_t waves = n * ws.G;
        const int gw = (int)std::max<int64_t>(1, std::min<int64_t>((waves + 3) / 4, 32768));
        ProfScope _ps("k_ds_filter", st);
        hipLaunchKernelGGL((k_ds_filter<16>), dim3(gw), dim3(256), 0, st, rows, n, d, ws);
    }
    FLC_CHECK_LAUNCH("k_ds_filter");
    hipLaunchKernelGGL(k_ds_final, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, n, ws, w, pnorm_out);
    FLC_CHECK_LAUNCH("k_ds_final");
    {
        const int ab = (int)std::max<int64_t>(1, std::min<int64_t>((C + 3) / 4, 4096));
        ProfScope _ps("k_ds_accum", st);
        if (w) hipLaunchKernelGGL((k_ds_accum<true>), dim3(ab), dim3(256), 0, st, rows, n, d, ws, prm->d_levels, prm->s, w, wt, out);
        else hipLaunchKernelGGL((k_ds_accum<false>), dim3(ab), dim3(256), 0, st, rows, n, d, ws, prm->d_levels, prm->s, w, wt, out);
    }
    FLC_CHECK_LAUNCH("k_ds_accum");
    return FLC_OK;
}

}  // namespace flc
