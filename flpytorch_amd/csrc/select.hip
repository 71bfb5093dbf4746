// Sparsifying codecs: TopK (compressors.py:330-335) and RandK (240-245), dense single-vector
// encode and fused batch encode + reduce.
//
// Data flow of the batch path (N client rows x D, chunk = 4096 elements = one wave's tile):
//
//   TopK  sample   : one workgroup per row keys a spread sample (<= 16 K elements, LDS) and picks a
//                    conservative threshold T_lo with count(|x| >= T_lo) >= K w.h.p.
//         filter   : ONE pass over every row (the only full HBM read): entries with key >= T_lo
//                    are appended to the row's candidate list (idx, val), per chunk -> tab[c][row]
//         select   : exact K-th largest key among the candidates (3 radix passes, 11/11/9 bits)
//         fallback : rows whose list overflowed, came up short (sample unlucky), or whose K-th
//                    magnitude is tied ambiguously are redone exactly on the full row
//                    (3 radix passes + tie prefix + exact filter, ties -> lowest index first)
//   RandK device   : the device sampler (randk_tree.hpp) is generated chunk by chunk: per row the
//                    chunk counts (k_randk_counts, a hypergeometric tree), then one wave per chunk
//                    regenerates every row's members of its chunk, gathers (D/K) * x[j] and folds
//                    them in row order (k_randk_fold) — no index lists in memory; the only HBM
//                    traffic is the gathered 128-B lines and the [D] result
//   RandK compat   : the K numpy-stream indices of each row are bucketed by chunk in two coalesced
//                    levels — superchunks in one workgroup per row (LDS counts + multi-split),
//                    then chunks inside each superchunk (LDS counting sort) with the gather of
//                    (D/K) * x[j] in ascending order (k_randk_coarse / k_randk_fine)
//   accumulate     : one wave owns one chunk (or 1/2, 1/4 of it when the rows are short) as an
//                    fp32 LDS tile and folds the rows' admitted
//                    entries in row order -> (sum_i w_i C_i(x_i)) / w_total, bit-identical to the
//                    sequential reduction of the dense compressVector outputs (indices are
//                    distinct within a row, so every element sees its terms in row order).
//
// Keys: |x| bits with the sign cleared (uint32, monotone; NaN above inf like torch.topk).
#include <stdlib.h>

#include <atomic>
#include <map>
#include <mutex>
#include <vector>

#include "chunks.hpp"
#include "randk_tree.hpp"

namespace flc {

constexpr uint32_t ALL = 0xFFFFFFFFu;
constexpr uint32_t F_OVERFLOW = 1u, F_SHORT = 2u, F_TIES = 4u, F_EXACT = 8u;
constexpr uint32_t F_RESIDENT = 16u;  // a lone row selected exactly in registers (k_lone_resident)
constexpr uint32_t F_REPAIR = 32u;    // ... whose grid was not co-resident: re-selected by its last workgroup
constexpr int SMAX = 16384;          // sample size kept in LDS
constexpr int HBINS = 2048;          // radix histogram bins (11 bits)
constexpr uint32_t TIECAP = HBINS;   // fast-path tie list (LDS); more ties at the K-th key -> exact path
constexpr int CS_SH = 64;            // few rows: shards of a row's candidate list (k_cs_pass workgroups)
constexpr int64_t CS_FEW = 16;       // rows: sharded lists + k_cs_pass up to here, else k_cand_select
constexpr int CS_ST = 8;             // words of a row's k_cs_pass state
constexpr int CS_LCAP = 2048;        // entries of the first digit's bin ranked directly (list mode)
constexpr int RS_U = 16;             // (<= 16: kept-tie mask of 64 bits) k_lone_resident: float4 of the row per thread at most (64 VGPRs)
#ifndef FLC_RS_NG
#define FLC_RS_NG 4                   // k_lone_resident: workgroup groups (histogram replicas, barrier tree);
#endif                                // us a call at D = 10 M: 1 -> 57, 2 -> 53, 4 -> 52, 8 -> 54.6, 16 -> 60
constexpr int RS_NG = FLC_RS_NG;
constexpr int RS_NG_MAX = 16;
static_assert(RS_NG >= 1 && RS_NG <= RS_NG_MAX, "FLC_RS_NG: 1..16 groups");
// its control words: counters on lines of their own, per-group digit histograms, tie counts
// (RS_GAVE: the sequence number of a call that was aborted; RS_XGRP: workgroups that have left)
constexpr int RS_GLOB = 0, RS_GEN = 32, RS_GAVE = 64, RS_CCNT = 96, RS_CDONE = 112, RS_GRP = 128;
constexpr int RS_XGRP = RS_GRP + 32 * RS_NG_MAX;  // per group: workgroups counted out (runs on across calls)
constexpr int RS_ABV = RS_XGRP + 32 * RS_NG_MAX;   // per group: keys above the speculated first digits
constexpr int RS_CAP = 2048;          // candidates (22-bit prefix of the K-th key) ranked by the last workgroup
constexpr int RS_SS = 8192;           // the speculative first digit's sample (32 pieces of 256)
#ifndef FLC_RS_SR
#define FLC_RS_SR 1                   // replicas of the sample's histogram (LDS; 8 measured 0.35 us slower a call)
#endif
constexpr int RS_SR = FLC_RS_SR;
#ifndef FLC_RS_STPOL
#define FLC_RS_STPOL 2                // the dense output's stores: nontemporal (2) or default (0)
#endif
#ifndef FLC_RS_GACQ
#define FLC_RS_GACQ 1                 // k_lone_resident: a group's last arriver acquires before its release
#endif
#ifndef FLC_RS_POLLAB
#define FLC_RS_POLLAB 1               // k_lone_resident: a grid wait reads the abort word every n-th poll
#endif
#ifndef FLC_RS_DONE
// k_lone_resident's candidate hand-over: 1 = a workgroup holding candidates reserves their place in
// the shared list (one returning add), stores them and then adds their number to a delivered count;
// the ranking workgroup waits for that count to reach the candidates' total (known to all from the
// round's payload), not for every workgroup to count out, and reads the list in one pass.
// 0 = per-workgroup slots gathered after every workgroup counted out.
#define FLC_RS_DONE 1
#endif
#ifndef FLC_RS_RANKFIRST
#define FLC_RS_RANKFIRST 0            // 1: the ranking workgroup ranks before its own dense stores (measured 0.2 us slower)
#endif
#ifndef FLC_RS_PROBE_NOCOUNT
#define FLC_RS_PROBE_NOCOUNT 0        // (cost probes only: no exit count — an aborted call would not repair)
#endif
#ifndef FLC_RS_G0REL
#define FLC_RS_G0REL 1                // workgroup 0 releases the row state before it counts out
#endif
#ifndef FLC_RS_FENCE
// k_lone_resident's grid rounds: 1 = agent-scope release / acquire fences around the counters (an
// L2 write-back or L1 invalidate each, ~1.7 us; five on the last arriver's path); 0 = no fences —
// every byte handed over inside the launch is written by an agent-scope atomic (histogram adds,
// list entries, counters, the release word) and read by agent-scope (sc1) loads, every writing
// wave drains (vmcnt(0)) before its workgroup's one counter add, and the counters never need a
// reset store (see rs_arrive)
#define FLC_RS_FENCE 0
#endif
#ifndef FLC_RS_SPEC
#define FLC_RS_SPEC 1                 // k_lone_resident: speculative first digit (two digits in one round)
#endif
constexpr int RS_HREP = RS_ABV + 32 * RS_NG_MAX;
constexpr int RS_HSPEC = RS_HREP + 3 * RS_NG * HBINS;    // [RS_NG][3][HBINS] speculative second digit
constexpr int RS_CLIST = RS_HSPEC + 3 * RS_NG * HBINS;   // [RS_CAP] (value bits, index)
constexpr int RS_TCNT = RS_CLIST + 2 * RS_CAP;               // (tie counts: 64-bit (call << 32 | count) per workgroup)
constexpr int RS_GMAX = 1024;                                  // workgroups a launch may have (tie counts, list slots)
constexpr int RS_CS = 4;                                       // listed elements a workgroup keeps in slots of its own
constexpr int RS_CNUM = RS_TCNT + 2 * RS_GMAX;                 // [RS_GMAX] elements a workgroup listed (this call)
constexpr int RS_CREG = RS_CNUM + RS_GMAX;                     // [RS_GMAX][RS_CS] 64-bit (value bits, index)
#ifdef FLC_RS_PRINT
constexpr int RS_PROBE = RS_CREG + 2 * RS_CS * RS_GMAX;        // probe builds: per-workgroup phase stamps
constexpr int RS_CTL = RS_PROBE + 4096;
#else
constexpr int RS_CTL = RS_CREG + 2 * RS_CS * RS_GMAX;
#endif
#ifndef FLC_RS_SPECST
#define FLC_RS_SPECST 0               // 1: the dense output outside the speculative window stored during the round (slower: 42.5 vs 36.7 us, the writes delay the merger)
#endif
#ifndef FLC_CS_LIST
#define FLC_CS_LIST 1
#endif
#ifndef FLC_CS_TWO_MAXD
#define FLC_CS_TWO_MAXD (int64_t(64) << 20)   // rows up to this long: two k_cs_pass launches
#endif

struct SelWs {            // carved from the caller workspace
    uint2* tab;           // [C][N] (offset, count) of each row's entries in chunk c
    uint32_t* ent_idx;    // [N][cap] element index within the row
    float* ent_val;       // [N][cap] entry value (already scaled for RandK)
    uint32_t* rowcnt;     // [N * RCS] entries used (one counter per 128 B line)
    uint32_t* flags;      // [N]
    uint32_t* thr;        // [N] admission key: entries with key >= thr are summed
    uint32_t* prefix;     // [N] radix-select state
    uint32_t* krem;       // [N]
    uint32_t* tieprefix;  // [C][N] ties (key == thr) in chunks before c   (exact path only)
    uint32_t* tiecut;     // [N] fast path, F_TIES: the last index admitted among key == thr (tie_pref order);
                          // rows selected by k_radix_select<FULLROW> (dense K): the count of keys == thr
    uint32_t* hist;       // [N][HBINS]
    uint32_t* worklist;   // [N] rows on the exact path
    uint32_t* nwork;      // [1]
    uint32_t* cursor;     // [C][N] RandK scatter cursors
    uint32_t* cstate;     // [N][CS_ST] few-row candidate select: shift, prefix, krem, stage, bin count, list fill (k_cs_pass)
    uint64_t* clist;      // [min(N, CS_FEW)][CS_LCAP] few rows: the first digit bin's entries (k_cs_pass list mode)
    uint32_t* carrive;    // [N * RCS] its per-row arrival counters
    uint32_t* shcnt;      // [N][CS_SH * RCS] few rows: the filter's reservation counters, one per shard
    uint32_t* zm;         // [C][CHUNK / 32] k_chunk_accum (one-wave blocks): a fold job's kept-column mask
    float* part;          // [D] TopK row-group folds: the running tiles carried from one group to the next
    int64_t cap;
    uint32_t tie_hi;      // TopK ties at the K-th key: 0 the lowest indices are kept (default), 1 the highest
};

// Tie order of TopK (flc_codec_params.tie): tie_pref(ix) is larger for the index kept first among
// equal magnitudes — ~ix for the lowest-index rule (the oracle's, torch.topk's CPU order on the
// reference's rows), ix for the highest-index rule.  A row's tie cut is the last kept tie's index:
// a tie is admitted iff tie_pref(ix) >= tie_pref(cut); tie_all(ws) is the cut that admits every tie.
__device__ __host__ inline uint32_t tie_pref(uint32_t ix, uint32_t hi) { return hi ? ix : ~ix; }
__device__ __host__ inline uint32_t tie_all(uint32_t hi) { return hi ? 0u : 0xFFFFFFFFu; }


// ------------------------------------------------------------------------------------------
// Block-level helpers
// ------------------------------------------------------------------------------------------
// Find, scanning a 2048-bin histogram from the TOP bin down, the bin b where the running count
// reaches k (1-based).  Returns b and the count strictly above b.  256 threads, 8 bins each.
// (t, own): the thread's index in the 256 that scan; every thread of the block takes the barriers.
// A workgroup barrier for LDS only: this wave's LDS operations done, then s_barrier — unlike
// __syncthreads it does not wait for the wave's global loads (vmcnt), so loads stay in flight.
__device__ inline void lds_bar() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}
template <bool RAW>
__device__ inline void blk_bar() {
    if (RAW) lds_bar();
    else __syncthreads();
}
template <bool RAW = false>
__device__ inline void hist_find_at(const uint32_t* h, uint32_t k, uint32_t& bin, uint32_t& above,
                                    uint32_t* scratch /* LDS 256+2 */, int t, bool own) {
    // thread t owns bins [HBINS-8(t+1), HBINS-8t)  (top bins first)
    uint32_t local[8];
    uint32_t s = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) { local[q] = own ? h[HBINS - 1 - (t * 8 + q)] : 0u; s += local[q]; }
    if (t == 0) { scratch[256] = 0; scratch[257] = 0; }   // defined result even if k > total
    // inclusive scan over the 256 thread sums: inside each wave by shuffles, then the totals of the
    // waves before (one barrier instead of the 16 of a Hillis-Steele scan through LDS)
    const int lane = t & 63, w = t >> 6;
    uint32_t inc = s;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = __shfl_up(inc, off, 64);
        inc += lane >= off ? v : 0u;
    }
    if (own && lane == 63) scratch[w] = inc;
    blk_bar<RAW>();
    uint32_t before = 0;
    if (own)
        for (int q = 0; q < w; ++q) before += scratch[q];
    uint32_t incl = own ? before + inc : 0u, excl = incl - s;
    if (own && excl < k && incl >= k) {
        uint32_t run = excl;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            if (run + local[q] >= k) {
                scratch[256] = (uint32_t)(HBINS - 1 - (t * 8 + q));
                scratch[257] = run;
                break;
            }
            run += local[q];
        }
    }
    blk_bar<RAW>();
    bin = scratch[256];
    above = scratch[257];
    blk_bar<RAW>();
}
// The same search over NB bins (NB / 256 a thread, threads 0..255 of a larger block; the rest only
// sync); found = false when the bins hold fewer than k in all.
template <int NB>
__device__ inline void hist_find_n(const uint32_t* h, uint32_t k, uint32_t& bin, uint32_t& above, bool& found,
                                   uint32_t* scratch /* LDS 256+3 */) {
    constexpr int PER = NB / 256;
    static_assert(NB % 256 == 0, "256 threads scan NB / 256 bins each");
    const int t = (int)threadIdx.x;
    const bool own = t < 256;
    uint32_t local[PER];
    uint32_t s = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) { local[q] = own ? h[NB - 1 - (t * PER + q)] : 0u; s += local[q]; }
    if (t == 0) { scratch[256] = 0; scratch[257] = 0; scratch[258] = 0; }
    const int lane = t & 63, w = t >> 6;
    uint32_t inc = s;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = __shfl_up(inc, off, 64);
        inc += lane >= off ? v : 0u;
    }
    if (own && lane == 63) scratch[w] = inc;
    __syncthreads();
    uint32_t before = 0;
    if (own)
        for (int q = 0; q < w; ++q) before += scratch[q];
    const uint32_t incl = own ? before + inc : 0u, excl = incl - s;
    if (own && excl < k && incl >= k) {
        uint32_t run = excl;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            if (run + local[q] >= k) {
                scratch[256] = (uint32_t)(NB - 1 - (t * PER + q));
                scratch[257] = run;
                scratch[258] = 1;
                break;
            }
            run += local[q];
        }
    }
    __syncthreads();
    bin = scratch[256];
    above = scratch[257];
    found = scratch[258] != 0u;
    __syncthreads();
}
template <bool RAW = false>
__device__ inline void hist_find(const uint32_t* h, uint32_t k, uint32_t& bin, uint32_t& above,
                                 uint32_t* scratch /* LDS 256+2 */) {
    hist_find_at<RAW>(h, k, bin, above, scratch, (int)threadIdx.x, threadIdx.x < 256);   // larger blocks: the rest only sync
}
// Two searches side by side (blocks of >= 512 threads): threads 0-255 scan ha for ka, 256-511 hb for kb.
__device__ inline void hist_find2(const uint32_t* ha, uint32_t ka, uint32_t& bina, uint32_t& abovea, uint32_t* sa,
                                  const uint32_t* hb, uint32_t kb, uint32_t& binb, uint32_t& aboveb, uint32_t* sb) {
    const bool second = threadIdx.x >= 256;
    uint32_t bin, above;
    hist_find_at(second ? hb : ha, second ? kb : ka, bin, above, second ? sb : sa, (int)(threadIdx.x & 255u),
                 threadIdx.x < 512);
    bina = sa[256]; abovea = sa[257];
    binb = sb[256]; aboveb = sb[257];
    __syncthreads();
}

// pass p: 0 -> bits [30:20], 1 -> [19:9], 2 -> [8:0]
__device__ inline uint32_t pass_shift(int p) { return p == 0 ? 20u : (p == 1 ? 9u : 0u); }
__device__ inline uint32_t pass_bits(int p) { return p == 2 ? 9u : 11u; }
__device__ inline bool key_in_prefix(uint32_t key, int p, uint32_t prefix) {
    // prefix holds the bits above this pass's field
    if (p == 0) return true;
    uint32_t sh = pass_shift(p) + pass_bits(p);
    return (key >> sh) == prefix;
}
__device__ inline uint32_t key_bin(uint32_t key, int p) {
    return (key >> pass_shift(p)) & ((1u << pass_bits(p)) - 1u);
}

// ------------------------------------------------------------------------------------------
// TopK: sample threshold (one workgroup per row)
// ------------------------------------------------------------------------------------------
// DUAL (few rows: latency-bound): the two rank searches share their passes over the sample; the
// second histogram costs 8 KB of LDS, which would halve the workgroups per CU of a many-row launch.
template <int NT, bool DUAL>
__global__ __launch_bounds__(NT) void k_topk_sample(RowSrc rows, int64_t n, int64_t d, int64_t K, SelWs ws, int few,
                                                    int64_t r_off) {
    __shared__ uint32_t keys[SMAX];
    __shared__ uint32_t h[HBINS], h2[DUAL ? HBINS : 1];
    __shared__ uint32_t scratch[260], scratch2[DUAL ? 260 : 1];
    const int64_t row = r_off + blockIdx.x;                               // (a launch may take a row range)
    if (row >= n) return;
    const float* r = rows.row(row);
    // sample: the whole row if it fits, else P pieces of 256 contiguous elements spread evenly
    int S;
    if (d <= SMAX) {
        S = (int)d;
        for (int i = threadIdx.x; i < S; i += NT) keys[i] = mag_key(r[i]);
    } else {
        const int P = SMAX / 256;
        S = SMAX;
        // piece p = 256 contiguous elements at p (d - 256) / (P - 1); thread t reads element t of
        // 32 pieces per round trip (a lone row's sample is latency-bound: few trips)
        // NT / 256 groups of threads take interleaved pieces
        constexpr int GR = NT / 256, PU = 32 / GR;
        const int e = threadIdx.x & 255, g0 = threadIdx.x >> 8;
        for (int p0 = 0; p0 < P; p0 += 32) {
            float x[PU];
#pragma unroll
            for (int u = 0; u < PU; ++u) x[u] = r[((int64_t)(p0 + u * GR + g0) * (d - 256)) / (P - 1) + e];
#pragma unroll
            for (int u = 0; u < PU; ++u) keys[(p0 + u * GR + g0) * 256 + e] = mag_key(x[u]);
        }
    }
    // a spread sample (S < d) only bounds the threshold: its keys to 22 bits (two passes, the low 9
    // bits 0: a lower bound, ~6e-5 relative below the key); the whole row (S == d) exactly
    const int NP = S == d ? 3 : 2;
    // rank (from the top) of the sample element whose key is the threshold
    uint32_t rank;
    if (S == d) {
        rank = (uint32_t)K;                                   // exact
    } else {
        double ks = (double)K * (double)S / (double)d;
        double rr = ks + 4.0 * sqrt(ks) + 8.0;
        rank = (uint32_t)min((double)S, ceil(rr));
    }
    // keys of sample ranks ra and rb (from the top) together: three 11/11/9-bit passes over the LDS
    // sample, one histogram while the two prefixes agree (always in the first pass), the two
    // searches side by side
    static_assert(!DUAL || NT >= 512, "hist_find2 takes 512 threads");
    auto rank_key = [&](uint32_t r) {
        uint32_t prefix = 0, krem = r;
        for (int p = 0; p < NP; ++p) {
            for (int i = threadIdx.x; i < HBINS; i += NT) h[i] = 0;
            __syncthreads();
            for (int i = threadIdx.x; i < S; i += NT) {
                uint32_t k = keys[i];
                if (key_in_prefix(k, p, prefix)) atomicAdd(&h[key_bin(k, p)], 1u);
            }
            __syncthreads();
            uint32_t bin, above;
            hist_find(h, krem, bin, above, scratch);
            prefix = (prefix << pass_bits(p)) | bin;
            krem -= above;
            __syncthreads();
        }
        return NP == 3 ? prefix : prefix << 9;
    };
    auto rank_keys = [&](uint32_t ra, uint32_t rb, uint32_t& ka, uint32_t& kb) {
        if constexpr (!DUAL) {
            ka = rank_key(ra);
            kb = rb == ra ? ka : rank_key(rb);
            return;
        }
        uint32_t pa = 0, pb = 0, ma = ra, mb = rb;
        for (int p = 0; p < NP; ++p) {
            const bool same = pa == pb;
            for (int i = threadIdx.x; i < HBINS; i += NT) { h[i] = 0; h2[i] = 0; }
            __syncthreads();
            for (int i = threadIdx.x; i < S; i += NT) {
                const uint32_t k = keys[i];
                if (key_in_prefix(k, p, pa)) atomicAdd(&h[key_bin(k, p)], 1u);
                if (!same && key_in_prefix(k, p, pb)) atomicAdd(&h2[key_bin(k, p)], 1u);
            }
            __syncthreads();
            uint32_t ba, aa, bb, ab;
            hist_find2(h, ma, ba, aa, scratch, same ? h : h2, mb, bb, ab, scratch2);
            pa = (pa << pass_bits(p)) | ba;
            ma -= aa;
            pb = (pb << pass_bits(p)) | bb;
            mb -= ab;
        }
        ka = NP == 3 ? pa : pa << 9;
        kb = NP == 3 ? pb : pb << 9;
    };
    // the threshold key (rank), and the estimate of the K-th key (sample rank ks) that sizes the
    // first digit of k_cand_select
    uint32_t tkey, kest;
    rank_keys(rank, S == d ? rank : (uint32_t)max(1.0, min((double)S, (double)K * (double)S / (double)d)), tkey, kest);
    if (threadIdx.x == 0) {
        ws.thr[row] = (rank >= (uint32_t)S && S != d) ? 0u : tkey;
        ws.prefix[row] = kest;
        ws.flags[row] = 0;
        ws.rowcnt[(row) * RCS] = 0;
        if (few) { ws.cstate[row * CS_ST + 3] = 0; ws.cstate[row * CS_ST + 5] = 0; ws.carrive[row * RCS] = 0; }
    }
    if (few && threadIdx.x < CS_SH) ws.shcnt[(row * CS_SH + threadIdx.x) * RCS] = 0;
    if (few)                                              // the row's global histogram of k_cs_pass
        for (int i = threadIdx.x; i < HBINS; i += NT) ws.hist[row * HBINS + i] = 0;
}

// ------------------------------------------------------------------------------------------
// Exact K-th key over a row's candidate list (fast path), one workgroup per row.
// Every candidate has key >= T (the sample threshold), and the K-th largest key of the row is
// among them when the list holds >= K entries.  Digits are taken of the offset dk = key - T:
// the first digit is dk >> s0 clamped to HBINS-1, with s0 sized so that the sample's estimate of
// the K-th key falls in the lowest quarter of the bins; the following digits are 11-bit slices
// of dk below s0 (usually one, exact: 2 passes over the list instead of 3 full-key passes, and
// the bins spread over the populated range instead of the few exponent values a full-key first
// digit sees).  A K-th key in the clamp bin (estimate off by > 4x) sends the row to the exact
// path.  Result as k_radix_select's last pass: thr = K-th key, krem = ties to admit, F_TIES when
// the list has more keys equal to thr than that.
// ------------------------------------------------------------------------------------------
// candidate values of a row, read twice per launch (measured: nt loads 0.335 -> 0.293 ms at C3)
#ifndef FLC_CS_NT
#define FLC_CS_NT 1
#endif
__device__ inline float4 cs_ld(const float4* p) {
#if FLC_CS_NT
    typedef float v4f __attribute__((ext_vector_type(4)));
    const v4f v = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
#else
    return *p;
#endif
}
template <int NT>
__device__ void cand_select_row(int64_t row, int64_t K, SelWs ws, uint32_t* h, uint32_t* scratch) {
    {
        if (ws.flags[row]) return;                                       // overflowed in the filter
        const uint32_t cnt = ws.rowcnt[(row) * RCS];
        if (cnt < (uint32_t)K) {                                          // sample threshold too high
            if (threadIdx.x == 0) ws.flags[row] |= F_SHORT;
            return;
        }
        const uint32_t T = ws.thr[row];
        const uint32_t span = ws.prefix[row] - T;                         // kest >= T
        int s = 0;
        while (s < 21 && (((uint64_t)span * 4u) >> s) >= (uint64_t)HBINS) ++s;
        const float* vals = ws.ent_val + row * ws.cap;                    // cap % 4 == 0: 16 B rows
        const float4* v4 = reinterpret_cast<const float4*>(vals);
        const uint32_t n4 = cnt >> 2;
        uint32_t prefix = 0, krem = (uint32_t)K, last = 0;
        bool first = true, fail = false;
        int sh = s;
        while (true) {
            const int s1 = first ? sh : max(0, sh - 11);
            const uint32_t mask = first ? 0xFFFFFFFFu : ((1u << (sh - s1)) - 1u);
            for (int i = threadIdx.x; i < HBINS; i += NT) h[i] = 0;
            __syncthreads();
            auto add = [&](float x) {
                const uint32_t dk = mag_key(x) - T;
                if (first) atomicAdd(&h[min(dk >> s1, (uint32_t)(HBINS - 1))], 1u);
                else if ((dk >> sh) == prefix) atomicAdd(&h[(dk >> s1) & mask], 1u);
            };
            // 8 float4 per thread in flight per round trip (the walk is latency-bound otherwise)
            uint32_t i = threadIdx.x;
            for (; i + 7 * NT < n4; i += 8 * NT) {
                float4 q[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) q[u] = cs_ld(v4 + i + u * NT);
#pragma unroll
                for (int u = 0; u < 8; ++u) { add(q[u].x); add(q[u].y); add(q[u].z); add(q[u].w); }
            }
            for (; i < n4; i += NT) {
                const float4 q = v4[i];
                add(q.x); add(q.y); add(q.z); add(q.w);
            }
            for (uint32_t i = n4 * 4 + threadIdx.x; i < cnt; i += NT) add(vals[i]);
            __syncthreads();
            uint32_t bin, above;
            hist_find(h, krem, bin, above, scratch);
            last = h[bin];
            if (first && bin == HBINS - 1) { fail = true; break; }
            prefix = first ? bin : ((prefix << (sh - s1)) | bin);
            krem -= above;
            sh = s1;
            first = false;
            __syncthreads();
            if (sh == 0) break;
        }
        __syncthreads();
        // ambiguous ties (more entries with key == thr than places left): the reference keeps the
        // lowest indices (torch.topk on CPU; oracle.codecs.topk_indices).  Gather the tie indices
        // and find the krem-th smallest: the admission cut for k_chunk_accum.
        const uint32_t thr = T + prefix;
        bool ties = !fail && last > krem;
        if (ties && last > TIECAP) { fail = true; ties = false; }      // pathological: exact path
        if (ties) {
            uint32_t* tix = h;                                           // reuse the histogram
            if (threadIdx.x == 0) scratch[0] = 0;
            __syncthreads();
            const uint32_t* idxs = ws.ent_idx + row * ws.cap;
            for (uint32_t i = threadIdx.x; i < n4; i += NT) {
                const float4 q = v4[i];
                const float qv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (mag_key(qv[u]) == thr) tix[atomicAdd(&scratch[0], 1u)] = idxs[i * 4 + u];
            }
            for (uint32_t i = n4 * 4 + threadIdx.x; i < cnt; i += NT) {
                if (mag_key(vals[i]) == thr) tix[atomicAdd(&scratch[0], 1u)] = idxs[i];
            }
            __syncthreads();
            const uint32_t m = scratch[0];                              // == last
            for (uint32_t a = threadIdx.x; a < m; a += NT) {
                const uint32_t ia = tix[a];
                uint32_t rank = 0;
                for (uint32_t b = 0; b < m; ++b) rank += tie_pref(tix[b], ws.tie_hi) > tie_pref(ia, ws.tie_hi) ? 1u : 0u;
                if (rank == krem - 1) ws.tiecut[row] = ia;              // indices are distinct
            }
        }
        if (threadIdx.x == 0) {
            if (fail) {
                ws.flags[row] |= F_SHORT;
            } else {
                ws.thr[row] = thr;
                ws.krem[row] = krem;
                if (ties) ws.flags[row] |= F_TIES;
            }
        }
        __syncthreads();
    }
}

template <int NT>
__global__ __launch_bounds__(NT) void k_cand_select(int64_t r0, int64_t rn, int64_t K, SelWs ws) {
    __shared__ uint32_t h[HBINS];
    __shared__ uint32_t scratch[260];
    for (int64_t row = r0 + blockIdx.x; row < r0 + rn; row += gridDim.x) {
        cand_select_row<NT>(row, K, ws, h, scratch);
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------
// The same selection for a few rows (a lone compressVector), spread over the chip: each row's
// list is split over gridDim.x workgroups that histogram their slices (LDS) into the row's global
// histogram (atomics); the last workgroup to arrive picks the digit (the same digits, bins and
// results as k_cand_select) and leaves the row's state for the next launch — one launch per digit
// instead of one latency-bound workgroup walking 1.4 K candidates twice.  Ambiguous ties at the
// K-th key (more entries equal to it than places left; ~1 row in 8 at D = 10 M) are resolved by the
// last arriver as k_cand_select does: the tie indices gathered over all shards, the krem-th smallest
// is the admission cut (the reference keeps the lowest indices).  Only more than TIECAP ties take
// the exact path.
// ------------------------------------------------------------------------------------------
constexpr int CS_NT = 256;
// final_pass: no launch follows this one (a row the digits have not settled by then takes the exact
// path); list mode (second pass, the first digit's bin holding at most CS_LCAP entries): every
// workgroup copies its shard's entries of that bin to the row's list and the last arriver ranks them
// by (key desc, index asc) — the K-th key and the tie cut at once, whatever bits are left below the
// first digit, so two launches settle the row.
__global__ __launch_bounds__(CS_NT) void k_cs_pass(int64_t K, SelWs ws, int final_pass) {
    __shared__ uint32_t h[HBINS];
    __shared__ uint32_t scratch[260];
    __shared__ uint32_t last_wg;
    __shared__ uint64_t lst[FLC_CS_LIST ? CS_LCAP : 1];
    const int64_t row = blockIdx.y;
    const uint32_t B = gridDim.x, b = blockIdx.x;
    uint32_t* cs = ws.cstate + row * CS_ST;                              // shift, prefix, krem, stage, bin count, list fill
    const uint32_t stage = cs[3];
    if (stage >= 2u) return;                                             // done: the whole grid row
    // the row's list is CS_SH shards (the filter's reservations): workgroup b walks shard b
    const uint32_t* shc = ws.shcnt + row * CS_SH * RCS;
    uint32_t cnt = 0;
    for (int k = 0; k < CS_SH; ++k) cnt += shc[k * RCS];
    const uint32_t mycnt = shc[b * RCS];
    const bool first = stage == 0u;
    if (first && (ws.flags[row] != 0u || cnt < (uint32_t)K)) {          // overflowed / sample too high
        if (b == 0 && threadIdx.x == 0) {
            if (ws.flags[row] == 0u) ws.flags[row] = F_SHORT;
            cs[3] = 2u;
        }
        return;
    }
    const uint32_t T = ws.thr[row];
    uint32_t sh, prefix, krem;
    if (first) {
        const uint32_t span = ws.prefix[row] - T;                        // kest >= T
        uint32_t s0 = 0;
        while (s0 < 21 && (((uint64_t)span * 4u) >> s0) >= (uint64_t)HBINS) ++s0;
        sh = s0; prefix = 0; krem = (uint32_t)K;
    } else {
        sh = cs[0]; prefix = cs[1]; krem = cs[2];
    }
    const uint32_t s1 = first ? sh : (sh > 11u ? sh - 11u : 0u);
    const uint32_t mask = first ? 0xFFFFFFFFu : ((1u << (sh - s1)) - 1u);
    const int64_t segcap = (ws.cap / CS_SH) & ~int64_t(3);
    if (FLC_CS_LIST && !first && cs[4] <= (uint32_t)CS_LCAP) {
        // list mode: this shard's entries of the first digit's bin, as (key << 32 | ~index)
        if (threadIdx.x == 0) scratch[0] = 0;
        __syncthreads();
        const float* sv = ws.ent_val + row * ws.cap + b * segcap;
        const uint32_t* si = ws.ent_idx + row * ws.cap + b * segcap;
        for (uint32_t e = threadIdx.x; e < mycnt; e += CS_NT) {
            const uint32_t key = mag_key(sv[e]);
            if (((key - T) >> sh) == prefix) {
                const uint32_t slot = atomicAdd(&scratch[0], 1u);
                if (slot < (uint32_t)CS_LCAP) lst[slot] = ((uint64_t)key << 32) | (uint64_t)tie_pref(si[e], ws.tie_hi);
            }
        }
        __syncthreads();
        const uint32_t nl = min(scratch[0], (uint32_t)CS_LCAP);
        if (threadIdx.x == 0) scratch[1] = nl ? atomicAdd(&cs[5], nl) : 0u;
        __syncthreads();
        uint64_t* gl = ws.clist + row * CS_LCAP;
        const uint32_t gb = scratch[1];
        for (uint32_t i = threadIdx.x; i < nl; i += CS_NT)
            if (gb + i < (uint32_t)CS_LCAP) gl[gb + i] = lst[i];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            last_wg = atomicAdd(&ws.carrive[row * RCS], 1u) == B - 1u ? 1u : 0u;
        }
        __syncthreads();
        if (!last_wg) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        const uint32_t m = __hip_atomic_load(&cs[5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool ok = m == cs[4] && m >= krem && krem >= 1u;          // every entry of the bin arrived
        const uint32_t mm = min(m, (uint32_t)CS_LCAP);
        for (uint32_t i = threadIdx.x; i < mm; i += CS_NT)
            lst[i] = __hip_atomic_load(&gl[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (threadIdx.x == 0) { scratch[0] = 0; scratch[1] = 0; scratch[2] = 0; scratch[3] = 0; }
        __syncthreads();
        // the entry of rank krem - 1 is the K-th: its key the threshold, its index the tie cut
        if (ok)
            for (uint32_t i = threadIdx.x; i < mm; i += CS_NT) {
                const uint64_t me = lst[i];
                uint32_t rank = 0;
                for (uint32_t j = 0; j < mm; ++j) rank += lst[j] > me ? 1u : 0u;
                if (rank == krem - 1u) { scratch[0] = (uint32_t)(me >> 32); scratch[1] = tie_pref((uint32_t)me, ws.tie_hi); }
            }
        __syncthreads();
        const uint32_t kth = scratch[0];
        if (ok)
            for (uint32_t i = threadIdx.x; i < mm; i += CS_NT) {
                const uint32_t key = (uint32_t)(lst[i] >> 32);
                if (key > kth) atomicAdd(&scratch[2], 1u);
                else if (key == kth) atomicAdd(&scratch[3], 1u);
            }
        __syncthreads();
        if (threadIdx.x == 0) {
            atomicExch(&ws.carrive[row * RCS], 0u);
            if (!ok) {
                ws.flags[row] |= F_SHORT;                                // exact path
            } else {
                const uint32_t gt = scratch[2], eq = scratch[3];
                ws.thr[row] = kth;
                ws.krem[row] = krem - gt;                                // ties admitted
                if (gt + eq > krem) { ws.tiecut[row] = scratch[1]; ws.flags[row] |= F_TIES; }
            }
            cs[3] = 2u;
        }
        return;
    }
    for (int i = threadIdx.x; i < HBINS; i += CS_NT) h[i] = 0;
    __syncthreads();
    auto add = [&](float x) {
        const uint32_t dk = mag_key(x) - T;
        if (first) atomicAdd(&h[min(dk >> s1, (uint32_t)(HBINS - 1))], 1u);
        else if ((dk >> sh) == prefix) atomicAdd(&h[(dk >> s1) & mask], 1u);
    };
    const float* vals = ws.ent_val + row * ws.cap + b * segcap;          // 16 B aligned shards
    const float4* v4 = reinterpret_cast<const float4*>(vals);
    const uint32_t n4 = mycnt >> 2, q1 = n4;
    uint32_t i = threadIdx.x;
    for (; i + 3 * CS_NT < q1; i += 4 * CS_NT) {
        float4 q[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) q[u] = cs_ld(v4 + i + u * CS_NT);
#pragma unroll
        for (int u = 0; u < 4; ++u) { add(q[u].x); add(q[u].y); add(q[u].z); add(q[u].w); }
    }
    for (; i < q1; i += CS_NT) {
        const float4 q = cs_ld(v4 + i);
        add(q.x); add(q.y); add(q.z); add(q.w);
    }
    for (uint32_t t = n4 * 4 + threadIdx.x; t < mycnt; t += CS_NT) add(vals[t]);
    __syncthreads();
    uint32_t* gh = ws.hist + row * HBINS;
    for (int t = threadIdx.x; t < HBINS; t += CS_NT)
        if (h[t]) atomicAdd(gh + t, h[t]);
    // publish: every wave's adds complete, then one release + the arrival (the last arriver picks)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last_wg = atomicAdd(&ws.carrive[row * RCS], 1u) == B - 1u ? 1u : 0u;
    }
    __syncthreads();
    if (!last_wg) return;
    // the row's histogram read and cleared with memory-side atomics: current on any XCD
    for (int t = threadIdx.x; t < HBINS; t += CS_NT) h[t] = atomicExch(gh + t, 0u);
    __syncthreads();
    uint32_t bin, above;
    hist_find(h, krem, bin, above, scratch);
    const uint32_t last = h[bin];
    const uint32_t np = first ? bin : ((prefix << (sh - s1)) | bin);
    const uint32_t nk = krem - above;
    const bool clamp = first && bin == HBINS - 1;                        // K-th key in the clamp bin
    bool ties = !clamp && s1 == 0u && last > nk, tie_fail = ties && last > TIECAP;
    if (ties && !tie_fail) {
        // gather the indices of the entries with key == thr over all shards (4 threads per shard,
        // 8 float4 per thread in flight), then the nk-th smallest index is the cut
        static_assert(CS_NT == 4 * CS_SH, "tie gather: 4 threads per shard");
        __syncthreads();                                                 // h[bin] read by every thread
        uint32_t* tix = h;
        if (threadIdx.x == 0) scratch[0] = 0;
        __syncthreads();
        const uint32_t thr = T + np;
        const int k = threadIdx.x >> 2;
        const uint32_t sub = threadIdx.x & 3u, c = shc[k * RCS], c4 = c >> 2;
        const float* sv = ws.ent_val + row * ws.cap + k * segcap;
        const uint32_t* si = ws.ent_idx + row * ws.cap + k * segcap;
        const float4* s4 = reinterpret_cast<const float4*>(sv);
        auto test = [&](float x, uint32_t pos) {
            if (mag_key(x) == thr) {
                const uint32_t slot = atomicAdd(&scratch[0], 1u);
                if (slot < TIECAP) tix[slot] = si[pos];
            }
        };
        uint32_t j = sub;
        for (; j + 28u < c4; j += 32u) {
            float4 q[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) q[u] = cs_ld(s4 + j + 4u * u);
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint32_t p4 = (j + 4u * u) * 4u;
                test(q[u].x, p4); test(q[u].y, p4 + 1u); test(q[u].z, p4 + 2u); test(q[u].w, p4 + 3u);
            }
        }
        for (; j < c4; j += 4u) {
            const float4 q = cs_ld(s4 + j);
            test(q.x, j * 4u); test(q.y, j * 4u + 1u); test(q.z, j * 4u + 2u); test(q.w, j * 4u + 3u);
        }
        for (uint32_t t = c4 * 4u + sub; t < c; t += 4u) test(sv[t], t);
        __syncthreads();
        const uint32_t m = scratch[0];                                   // == last
        if (m != last) tie_fail = true;                                  // (uniform: scratch[0] in LDS)
        else
            for (uint32_t a = threadIdx.x; a < m; a += CS_NT) {
                const uint32_t ia = tix[a];
                uint32_t rank = 0;
                for (uint32_t bb = 0; bb < m; ++bb) rank += tie_pref(tix[bb], ws.tie_hi) > tie_pref(ia, ws.tie_hi) ? 1u : 0u;
                if (rank == nk - 1u) ws.tiecut[row] = ia;                // indices are distinct
            }
    }
    if (threadIdx.x == 0) {
        atomicExch(&ws.carrive[row * RCS], 0u);
        if (clamp) {
            ws.flags[row] |= F_SHORT;
            cs[3] = 2u;
        } else if (s1 == 0u) {
            if (tie_fail) ws.flags[row] |= F_SHORT;                      // > TIECAP ties: exact path
            else {
                ws.thr[row] = T + np;
                ws.krem[row] = nk;
                if (ties) ws.flags[row] |= F_TIES;
            }
            cs[3] = 2u;
        } else if (final_pass) {
            ws.flags[row] |= F_SHORT;                                    // digits left, no launch: exact path
            cs[3] = 2u;
        } else {
            cs[0] = s1; cs[1] = np; cs[2] = nk; cs[3] = 1u; cs[4] = last;
        }
    }
}

// ------------------------------------------------------------------------------------------
// Filter: append entries with key >= thr (fast path) or the exact selection (exact path).
// One wave per chunk; a workgroup takes 4 chunks of one row; grid-stride over (row, 4-chunk).
// Exact mode (rows on the worklist, F_EXACT): key > thr always; key == thr only while the
// tie rank (tieprefix + rank in index order inside the chunk) < krem.
// ------------------------------------------------------------------------------------------
template <bool EXACT, bool VEC>
__global__ __launch_bounds__(256) void k_topk_filter(RowSrc rows, int64_t n, int64_t d, SelWs ws) {
    const int64_t C = nchunks(d);
    const int64_t bpr = (C + 3) / 4;                   // 4-chunk blocks per row
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t nrows = EXACT ? (int64_t)(*ws.nwork) : n;
    const int64_t items = nrows * bpr;
    for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
        const int64_t li = it / bpr;
        const int64_t row = EXACT ? (int64_t)ws.worklist[li] : li;
        const int64_t c = (it % bpr) * 4 + wv;
        if (!EXACT && ws.flags[row]) continue;          // already failed (row-uniform)
        if (c >= C) continue;
        const float* r = rows.row(row);
        const int64_t j0 = c * CHUNK;
        const uint32_t T = ws.thr[row];
        // load the chunk: 16 x float4 per lane, element j0 + (t*64 + lane)*4 + q
        float v[16][4];
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const int64_t j = j0 + (int64_t)(t * 64 + lane) * 4;
            if (VEC && j + 3 < d) {
                float4 f = *reinterpret_cast<const float4*>(r + j);
                v[t][0] = f.x; v[t][1] = f.y; v[t][2] = f.z; v[t][3] = f.w;
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) v[t][q] = (j + q < d) ? r[j + q] : 0.f;
            }
        }
        // ties (key == T) admitted: tie ranks [tie_from, tie_need) in index order — the first krem
        // (lowest-index rule) or the last krem of the row's tot (highest-index rule; k_radix_select
        // left tot in tiecut)
        uint32_t tie_base = 0, tie_need = ALL, tie_from = 0;
        if (EXACT) {
            tie_base = ws.tieprefix[c * n + row];
            tie_need = ws.krem[row];
            if (ws.tie_hi) { const uint32_t tot = ws.tiecut[row]; tie_from = tot - tie_need; tie_need = tot; }
        }
        // pass 1: count
        uint32_t cnt = 0;
        uint32_t tie_run = tie_base;
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const int64_t jb = j0 + (int64_t)(t * 64 + lane) * 4;
            bool gt[4], eq[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t k = mag_key(v[t][q]);
                const bool inb = (jb + q) < d;
                gt[q] = inb && (EXACT ? k > T : k >= T);
                eq[q] = inb && EXACT && k == T;
            }
            if (EXACT) {
                uint64_t m[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) m[q] = __ballot(eq[q]);
                const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
                uint32_t before = __popcll(m[0] & lt) + __popcll(m[1] & lt) + __popcll(m[2] & lt) + __popcll(m[3] & lt);
                uint32_t inlane = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (eq[q]) { const uint32_t tr = tie_run + before + inlane; gt[q] = tr >= tie_from && tr < tie_need; }
                    inlane += eq[q] ? 1u : 0u;
                }
                tie_run += __popcll(m[0]) + __popcll(m[1]) + __popcll(m[2]) + __popcll(m[3]);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) cnt += gt[q] ? 1u : 0u;
        }
        cnt = wave_sum(cnt);
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&ws.rowcnt[(row) * RCS], cnt);
        base = __shfl(base, 0, WAVE);
        const bool fits = (int64_t)base + cnt <= ws.cap;
        if (lane == 0) {
            ws.tab[c * n + row] = make_uint2(base, fits ? cnt : 0u);
            if (!fits) atomicOr(&ws.flags[row], F_OVERFLOW);
        }
        if (!fits || cnt == 0) continue;
        // pass 2: write (order inside the chunk is irrelevant to the result)
        uint32_t run = base;
        tie_run = tie_base;
        uint32_t* oi = ws.ent_idx + row * ws.cap;
        float* ov = ws.ent_val + row * ws.cap;
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const int64_t jb = j0 + (int64_t)(t * 64 + lane) * 4;
            bool gt[4], eq[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t k = mag_key(v[t][q]);
                const bool inb = (jb + q) < d;
                gt[q] = inb && (EXACT ? k > T : k >= T);
                eq[q] = inb && EXACT && k == T;
            }
            if (EXACT) {
                uint64_t m[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) m[q] = __ballot(eq[q]);
                const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
                uint32_t before = __popcll(m[0] & lt) + __popcll(m[1] & lt) + __popcll(m[2] & lt) + __popcll(m[3] & lt);
                uint32_t inlane = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (eq[q]) { const uint32_t tr = tie_run + before + inlane; gt[q] = tr >= tie_from && tr < tie_need; }
                    inlane += eq[q] ? 1u : 0u;
                }
                tie_run += __popcll(m[0]) + __popcll(m[1]) + __popcll(m[2]) + __popcll(m[3]);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint64_t m = __ballot(gt[q]);
                if (gt[q]) {
                    const uint32_t pos = run + (uint32_t)__popcll(m & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
                    oi[pos] = (uint32_t)(jb + q);
                    ov[pos] = v[t][q];
                }
                run += (uint32_t)__popcll(m);
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// Fast-path filter.  A work item is a group of GS consecutive 4096-element chunks of one row; waves
// walk items grid-stride.  Every chunk streams in through a RING-deep buffer-load pipeline that
// runs across chunk and item boundaries; entries with key >= T_lo are compacted (ballot / mbcnt)
// into a wave-private LDS staging buffer.  One atomic per group reserves the row-buffer space; its
// return is consumed only after the NEXT group has been compacted (double-buffered staging), when
// the group's entries are copied out coalesced and its GS tab entries are written.
//
// Why groups: on gfx950 vmcnt retires in order, so every atomic / store sits in front of the loads
// issued after it.  Per-chunk reservations (one atomic + a short copy-out per 4096 elements) cost
// ~20 % of the filter's bandwidth (tools/probe_filter.hip); a group of 4 amortises them 4x and the
// copy-out stores become full 256 B wave writes.
// ------------------------------------------------------------------------------------------
constexpr int GCAP = 512;             // staged entries per group (4 chunks: 3.1 %, ~2.5x the mean at 1.2 %; more -> row overflow)
static_assert(GCAP % 64 == 0, "copy-out runs in whole wave slots");


// A chunk is 16 wave-loads of 1 KB.  RING float4 registers per lane hold a software pipeline RING-1
// loads deep (the next chunk's descriptor is built up front; past the last item it has
// num_records 0 and its loads return zeros without touching memory).
// FGS: chunks per work item (group).
template <int RING, int FGS, int LONE = 0>
#ifndef FLC_TK_RING
#define FLC_TK_RING 16               // loads in flight per wave (ring registers: 4 x RING VGPRs)
#endif
#ifndef FLC_TK_STPOL
#define FLC_TK_STPOL 0               // A/B: the filter's list copy-out stores nontemporal (2) or default (0)
#endif
#ifndef FLC_TK_COPY4
#define FLC_TK_COPY4 1               // TopK filter copy-out: 16-B stores of whole quads
#endif
#ifndef FLC_TK_PROBE
#define FLC_TK_PROBE 0               // A/B cost probes (outputs NOT valid): 1 no staging writes, 2 no copy-out, 3 loads only
#endif
#ifndef FLC_TK_WPE
#define FLC_TK_WPE 1                 // unconstrained (143 VGPRs); 4 waves per SIMD spilled and ran slower
#endif
// LONE (a lone compressVector row on the list path): every float4 read is also written as zeros to
// zout, the dense output the selected entries are then scattered into (no separate fill of the output).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FLC_TK_WPE))) void k_topk_filter_fast(RowSrc rows, int64_t n, int64_t r0, int64_t rn, int64_t rb, int64_t d, SelWs ws, int shards,
                                                                                                float* __restrict__ zout) {
    static_assert(16 % RING == 0, "ring must divide the 16 loads of a chunk");
    // staging per (buffer, wave): GCAP + 64 indices then GCAP + 64 values (one ds_write2st64_b32
    // per entry; the 64 spare slots take a wave-instruction starting at GCAP, i.e. an overflow)
    constexpr int SROW = GCAP + 64;
    static_assert((SROW * 4) % 256 == 0, "value block offset in 256-byte units");
    __shared__ __attribute__((aligned(16))) uint32_t st[2][4][2 * SROW];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: keeps the item walk in SGPRs
    const int64_t C = nchunks(d);
    const int64_t G = (C + FGS - 1) / FGS;                               // groups per row
    const int64_t items = rn * G;                                        // this launch's rows: [r0, r0 + rn)
    const int64_t stride = (int64_t)gridDim.x * 4;
    int64_t it = (int64_t)blockIdx.x * 4 + wv;
    if (it >= items) return;
    float4 ring[RING];
    // item order: blocks of rb rows, inside a block (group, row) with the row fastest (rb = 1:
    // row-major)
    auto item_at = [&](int64_t t, int64_t& r, int64_t& cc) {
        const int64_t blk = t / (rb * G), rem = t - blk * rb * G;
        const int64_t bn = min(rb, rn - blk * rb);
        const int64_t g = rem / bn;
        r = r0 + blk * rb + (rem - g * bn);
        cc = g * FGS;
    };
    int64_t row, c;                                                      // current row, chunk
    item_at(it, row, c);
    auto rs = chunk_rsrc(rows.row_s(row), c * CHUNK, d);
#pragma unroll
    for (int L = 0; L < RING - 1; ++L) {
        ring[L] = load_q(rs, lane, L);
        __builtin_amdgcn_sched_barrier(0);   // issue in ring order: the loop's static vmcnt waits assume it
    }
    // few rows (shards > 1): group g of a row reserves in shard g % shards of its list (a counter and a
    // region of its own): one counter per row would serialise the reservation atomics of every
    // wave on one address (~90 per microsecond), a lone 10 M row's ~1.2 K of them took longer than
    // its loads
    const int64_t segcap = shards > 1 ? (ws.cap / shards) & ~int64_t(3) : ws.cap;
    // previous group, reservation in flight
    bool pv = false;
    int64_t prow = 0, pc0 = 0, pseg = 0;
    uint64_t pcc = 0;                        // per-chunk counts, 16 bits each
    uint32_t ptot = 0, pres = 0;
    int par = 0;
    auto finish = [&](int pb) {
        uint32_t base = 0;
        bool fits = ptot <= GCAP;
        if (fits && ptot) {
            base = __shfl(pres, 0, WAVE);
            fits = (int64_t)base + ptot <= segcap;
            base += (uint32_t)(pseg * segcap);                           // the shard's region
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
        if (!fits && lane == 0) atomicOr(&ws.flags[prow], F_OVERFLOW);
#if FLC_TK_COPY4
        {
            // Copy-out as 16-B stores of 4 entries a lane (the group's whole quads) plus the last
            // partial quad's entries as 4-B stores: a FIXED sequence of 2 GCAP / 256 + 2
            // range-checked buffer stores (none written when the group did not fit) instead of
            // 2 GCAP / 64 exec-masked 4-B stores — the copy-out cost the filter 0.5 ms of 6.9 per
            // C3 step (probe, same allocation).  The list position is any dword: the 16-B
            // stores need only dword alignment.
            const uint32_t* si = st[pb][wv];
            const uint32_t* sv = st[pb][wv] + SROW;
            const uint32_t nrec = (fits && FLC_TK_PROBE != 2) ? ptot * 4u : 0u;
            const auto di = __builtin_amdgcn_make_buffer_rsrc(ws.ent_idx + prow * ws.cap + base, (short)0, (int)nrec, 0x00020000);
            const auto dv = __builtin_amdgcn_make_buffer_rsrc(ws.ent_val + prow * ws.cap + base, (short)0, (int)nrec, 0x00020000);
            typedef unsigned int u4v __attribute__((ext_vector_type(4)));
            const uint32_t nq = ptot >> 2;
#pragma unroll
            for (int k = 0; k < GCAP / 256; ++k) {
                const uint32_t q = (uint32_t)(k * 64 + lane);
                const uint4 a = reinterpret_cast<const uint4*>(si)[q];
                const uint4 b = reinterpret_cast<const uint4*>(sv)[q];
                const uint32_t off = q < nq ? q * 16u : 0x7FFFFFF0u;
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, a), di, off, 0, FLC_TK_STPOL);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, b), dv, off, 0, FLC_TK_STPOL);
            }
            const uint32_t e = nq * 4u + (uint32_t)(lane & 3);          // the partial quad (range-checked)
            const uint32_t off = lane < 3 ? e * 4u : 0x7FFFFFF0u;
            __builtin_amdgcn_raw_buffer_store_b32(si[e], di, off, 0, FLC_TK_STPOL);
            __builtin_amdgcn_raw_buffer_store_b32(sv[e], dv, off, 0, FLC_TK_STPOL);
        }
#else
        if (fits && FLC_TK_PROBE != 2) {
            const uint32_t* si = st[pb][wv];
            const float* sv = reinterpret_cast<const float*>(st[pb][wv] + SROW);
            uint32_t* oi = ws.ent_idx + prow * ws.cap + base;
            float* ov = ws.ent_val + prow * ws.cap + base;
            // fixed trip count (GCAP / 64 predicated slots): the compiler's vmcnt bookkeeping
            // stays exact for the loads in flight behind these stores
#pragma unroll
            for (int k = 0; k < GCAP / 64; ++k) {
                const uint32_t e = (uint32_t)(k * 64 + lane);
                if (e < ptot) { oi[e] = si[e]; ov[e] = sv[e]; }
            }
        }
#endif
    };
    while (it < items) {
        // key >= max(T, 1): the loads past the row end return +0 (key 0), so no per-element range
        // test; a row whose K-th magnitude is 0 (fewer than K nonzeros) comes up short and takes
        // the exact path, which admits zeros
        const uint32_t T = max(sload(ws.thr + row), 1u);
        const int64_t nit = it + stride;
        // LDS byte address of this group's staging (wave-uniform)
        const uint32_t sla = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(__attribute__((address_space(3))) uint32_t*)st[par][wv]);
        uint32_t cnt = 0;                    // entries in this group so far
        uint64_t ccp = 0;
        const int64_t cg0 = c;
        int64_t nrow = row, nc = c;
        // straight-line over the group, no early exit: the chunks of a row's short last group
        // past the row end have empty descriptors (their loads return zeros), so the
        // compiler's vmcnt bookkeeping stays exact from one group's atomic to its use
#pragma unroll
        for (int sub = 0; sub < FGS; ++sub, ++c) {
            const int64_t j0 = c * CHUNK;
            // descriptor of the chunk after this one (same group, else the next item's first)
            __amdgpu_buffer_rsrc_t rsn;
            if (sub + 1 < FGS) {
                rsn = chunk_rsrc(rows.row_s(row), j0 + CHUNK, d);
            } else if (nit < items) {
                item_at(nit, nrow, nc);
                rsn = chunk_rsrc(rows.row_s(nrow), nc * CHUNK, d);
            } else {
                rsn = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(rows.row_s(row)), (short)0, 0, 0x00020000);
            }
            const uint32_t cnt0 = cnt;
            __amdgpu_buffer_rsrc_t ro;
            if constexpr (LONE != 0) ro = chunk_rsrc(zout, j0, d);
            // opaque per-chunk copy of the lane offset: stops LICM from hoisting the 64 per-(load,
            // component) index constants out of the loop into 64 live VGPRs
            uint32_t lb = (uint32_t)j0 + (uint32_t)lane * 4u;   // row index of the lane's element 0
            asm volatile("" : "+v"(lb));
#pragma unroll
            for (int L = 0; L < 16; ++L) {
                const int P = L + RING - 1;
                ring[P % RING] = P < 16 ? load_q(rs, lane, P) : load_q(rsn, lane, P - 16);
                const float4 x = ring[L % RING];
                if constexpr (LONE != 0) {
                    // unconditional (range-checked): one more store per step in the vmcnt queue
                    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
                    const u4v z = {0u, 0u, 0u, 0u};
                    __builtin_amdgcn_raw_buffer_store_b128(z, ro, lane * 16, L * 1024, 0);
                }
                const uint32_t jl = lb + (uint32_t)(L * 256);             // index in the row
                const float vq[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (FLC_TK_PROBE == 3) { cnt += __float_as_uint(vq[q]) == 0x7F800001u ? 1u : 0u; continue; }
                    const bool f = mag_key(vq[q]) >= T;
                    const uint64_t m = __ballot(f);
                    if (FLC_TK_PROBE != 1 && f) {
                        // slot = min(cnt, GCAP) + entries in lower lanes (< GCAP + 64): exact while
                        // the group fits; past GCAP it overflows (its row takes the exact path) and
                        // the writes land in the spare slots.  The scalar part folded into the LDS
                        // address in SALU, index and value out as one ds_write2st64_b32 (values
                        // SROW words on)
                        const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                        uint32_t sb = sla + min(cnt, (uint32_t)GCAP) * 4u;
                        asm volatile("" : "+s"(sb));
                        asm volatile("ds_write2st64_b32 %0, %1, %2 offset1:%3" ::"v"(sb + pre * 4u),
                                     "v"(jl + q), "v"(__float_as_uint(vq[q])), "i"(SROW * 4 / 256) : "memory");
                    }
                    cnt += (uint32_t)__popcll(m);
                }
            }
            ccp |= (uint64_t)min(cnt - cnt0, 0xFFFFu) << (16 * (c - cg0));
            rs = rsn;
        }
        if (pv) finish(par ^ 1);
        uint32_t res = 0;
        // the shard of the group's index within its row (the item order interleaves rows: `it % shards`
        // put each of n rows' items into only 64 / n shards, which overflowed them)
        const int64_t shard = shards > 1 ? (cg0 / FGS) % shards : 0;
        if (cnt && cnt <= GCAP && lane == 0)
            res = atomicAdd(shards > 1 ? &ws.shcnt[(row * shards + shard) * RCS] : &ws.rowcnt[(row) * RCS], cnt);
        pv = true; prow = row; pc0 = cg0; pcc = ccp; ptot = cnt; pres = res; pseg = shard;
        // the staging writes of this group and the copy-out reads of the buffer's next use are in
        // the wave's own program order; the fence keeps the compiler from moving LDS ops across
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
// Radix passes over candidate lists (fast path) or full rows (exact path)
// ------------------------------------------------------------------------------------------
// Histogram of pass p over row data; grid-stride over (row, block of 64 K elements).
template <bool FULLROW>
__global__ __launch_bounds__(256) void k_radix_hist(RowSrc rows, int64_t n, int64_t d, int p, SelWs ws) {
    __shared__ uint32_t h[HBINS];
    constexpr int64_t BLK = 65536;
    const int64_t nrows = FULLROW ? (int64_t)(*ws.nwork) : n;
    const int64_t maxlen = FULLROW ? d : ws.cap;
    const int64_t bpr = (maxlen + BLK - 1) / BLK;
    const int64_t items = nrows * bpr;
    for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
        const int64_t li = it / bpr;
        const int64_t row = FULLROW ? (int64_t)ws.worklist[li] : li;
        if (!FULLROW && ws.flags[row]) continue;
        const int64_t len = FULLROW ? d : (int64_t)ws.rowcnt[(row) * RCS];
        const int64_t b0 = (it % bpr) * BLK;
        if (b0 >= len) continue;
        const int64_t b1 = min(len, b0 + BLK);
        for (int i = threadIdx.x; i < HBINS; i += 256) h[i] = 0;
        __syncthreads();
        const uint32_t prefix = ws.prefix[row];
        const float* src = FULLROW ? rows.row(row) : (ws.ent_val + row * ws.cap);
        for (int64_t j = b0 + threadIdx.x; j < b1; j += 256) {
            const uint32_t k = mag_key(src[j]);
            if (key_in_prefix(k, p, prefix)) atomicAdd(&h[key_bin(k, p)], 1u);
        }
        __syncthreads();
        uint32_t* gh = ws.hist + row * HBINS;
        for (int i = threadIdx.x; i < HBINS; i += 256)
            if (h[i]) atomicAdd(&gh[i], h[i]);
        __syncthreads();
    }
}

// Select step of pass p: one workgroup per row.  After pass 2: thr = exact K-th key,
// krem = ties to admit.  Fast path: a short list (count < K) or ambiguous ties -> worklist.
template <bool FULLROW>
__global__ __launch_bounds__(256) void k_radix_select(int64_t n, int p, int64_t K, SelWs ws) {
    __shared__ uint32_t scratch[260];
    const int64_t nrows = FULLROW ? (int64_t)(*ws.nwork) : n;
    for (int64_t li = blockIdx.x; li < nrows; li += gridDim.x) {
        const int64_t row = FULLROW ? (int64_t)ws.worklist[li] : li;
        if (!FULLROW && ws.flags[row]) continue;
        uint32_t* gh = ws.hist + row * HBINS;
        if (!FULLROW && p == 0 && ws.rowcnt[(row) * RCS] < (uint32_t)K) {   // sample threshold too high
            for (int i = threadIdx.x; i < HBINS; i += 256) gh[i] = 0;
            if (threadIdx.x == 0) ws.flags[row] |= F_SHORT;
            continue;
        }
        const uint32_t k = (p == 0) ? (uint32_t)K : ws.krem[row];
        uint32_t bin, above;
        hist_find(gh, k, bin, above, scratch);
        const uint32_t ties_here = gh[bin];
        __syncthreads();
        for (int i = threadIdx.x; i < HBINS; i += 256) gh[i] = 0;    // ready for the next pass
        if (threadIdx.x == 0) {
            const uint32_t pre = (p == 0) ? 0u : ws.prefix[row];
            ws.prefix[row] = (pre << pass_bits(p)) | bin;
            ws.krem[row] = k - above;
            if (p == 2) {
                ws.thr[row] = ws.prefix[row];
                if (FULLROW) ws.tiecut[row] = ties_here;                  // the row's keys == thr (tie order)
                if (ties_here > k - above) ws.flags[row] |= (FULLROW ? F_TIES | F_EXACT : F_TIES);
                else if (FULLROW) ws.flags[row] |= F_EXACT;
            }
        }
        __syncthreads();
    }
}

// RowSrc that failed the fast path go on the worklist; their list state is reset.
__global__ void k_build_worklist(int64_t n, int64_t K, int64_t d, SelWs ws, int force_all) {
    // single block
    __shared__ uint32_t cnt;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    for (int64_t row = threadIdx.x; row < n; row += blockDim.x) {
        uint32_t f = ws.flags[row];
        if (force_all || (f & (F_OVERFLOW | F_SHORT))) {   // ambiguous ties stay on the fast path
            uint32_t pos = atomicAdd(&cnt, 1u);
            ws.worklist[pos] = (uint32_t)row;
            ws.flags[row] = F_EXACT;
            ws.rowcnt[(row) * RCS] = 0;
            ws.prefix[row] = 0;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) *ws.nwork = cnt;
}

// Exact path of the fast path's rare failures, in ONE launch: a workgroup per row (grid-stride),
// rows without F_OVERFLOW / F_SHORT return at once.  A failed row gets the exact radix select over
// its full row (three 11/11/9-bit passes, LDS histogram), then its list is rewritten chunk by
// chunk in index order: key > thr, plus the first krem elements with key == thr (the lowest
// indices, the oracle's tie rule), tab[c][row] = (offset, count), flags = F_EXACT (the fold admits
// the whole list).  The same selection as the multi-launch path (k_build_worklist, k_radix_*,
// k_tie_*, k_topk_filter<true>) that dense-K rows take, without its ~10 launches per call when no
// row failed.
constexpr int EX_NT = 1024;
constexpr int EX_U = 8;                      // float4 loads per thread in flight in the radix passes

// exclusive prefix of v over the workgroup's threads (in thread order) and the total
template <int NT = EX_NT>
__device__ inline uint32_t ex_scan(uint32_t v, uint32_t* wsum /* LDS [NT / 64] */, uint32_t& total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        inc += lane >= o ? t : 0u;
    }
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) {
        const uint32_t x = wsum[k];
        before += k < wv ? x : 0u;
        tot += x;
    }
    __syncthreads();
    total = tot;
    return before + inc - v;
}

// One row's exact selection by one EX_NT-thread workgroup: three radix passes over the row, then the
// row's list rewritten with exactly its admitted entries in index order (ties: the lowest indices).
template <bool VEC, int NT = EX_NT>
__device__ void exact_row(RowSrc rows, int64_t n, int64_t row, int64_t d, int64_t K, SelWs ws, uint32_t* h,
                          uint32_t* scratch, uint32_t* wsum) {
    const int t = threadIdx.x;
    const int64_t C = nchunks(d);
    {
        const float* r = rows.row(row);
        uint32_t prefix = 0, krem = (uint32_t)K, ties_tot = 0;
        for (int p = 0; p < 3; ++p) {
            for (int i = t; i < HBINS; i += NT) h[i] = 0;
            __syncthreads();
            auto add = [&](uint32_t k) { if (key_in_prefix(k, p, prefix)) atomicAdd(&h[key_bin(k, p)], 1u); };
            int64_t j = 0;
            if (VEC) {
                const float4* r4 = reinterpret_cast<const float4*>(r);
                const int64_t g4 = d / 4;
                int64_t g = t;
                for (; g + (EX_U - 1) * NT < g4; g += EX_U * NT) {
                    float4 q[EX_U];
#pragma unroll
                    for (int u = 0; u < EX_U; ++u) q[u] = ld_row4(r4 + g + u * NT);
#pragma unroll
                    for (int u = 0; u < EX_U; ++u) {
                        add(mag_key(q[u].x)); add(mag_key(q[u].y)); add(mag_key(q[u].z)); add(mag_key(q[u].w));
                    }
                }
                for (; g < g4; g += NT) {
                    const float4 q = ld_row4(r4 + g);
                    add(mag_key(q.x)); add(mag_key(q.y)); add(mag_key(q.z)); add(mag_key(q.w));
                }
                j = g4 * 4;
            }
            for (int64_t jj = j + t; jj < d; jj += NT) add(mag_key(r[jj]));
            __syncthreads();
            uint32_t bin, above;
            hist_find(h, krem, bin, above, scratch);
            prefix = (prefix << pass_bits(p)) | bin;                   // p == 0: prefix is 0
            krem -= above;
            if (p == 2) ties_tot = h[bin];                              // the row's keys == thr
            __syncthreads();
        }
        const uint32_t thr = prefix;                                    // the K-th key; krem ties admitted
        // tie ranks admitted in index order: [0, krem) (lowest-index rule) or [tot - krem, tot)
        const uint32_t tie_from = ws.tie_hi ? ties_tot - krem : 0u, tie_to = ws.tie_hi ? ties_tot : krem;
        uint32_t* oi = ws.ent_idx + row * ws.cap;
        float* ov = ws.ent_val + row * ws.cap;
        // a chunk is CHUNK / (NT * 4) sub-blocks of NT * 4 columns (1 for NT = 1024, 2 / 4 for the
        // 512 / 256-thread selects), walked in index order with base and tie_run carried across them
        static_assert(CHUNK % (NT * 4) == 0, "exact_row: NT * 4 must divide CHUNK");
        constexpr int SUBS = CHUNK / (NT * 4);
        uint32_t base = 0, tie_run = 0, cbase = 0;
        for (int64_t cs = 0; cs < C * SUBS; ++cs) {
            const int64_t c = cs / SUBS;
            const int sb = (int)(cs % SUBS);
            if (sb == 0) cbase = base;
            const int64_t j0 = c * CHUNK + (int64_t)sb * (NT * 4) + (int64_t)t * 4;
            float v[4];
            if (VEC && j0 + 3 < d) {
                const float4 q = ld_row4(reinterpret_cast<const float4*>(r + j0));
                v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = (j0 + q < d) ? r[j0 + q] : 0.f;
            }
            bool gt[4], eq[4];
            uint32_t ne = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bool in = j0 + q < d;
                const uint32_t k = mag_key(v[q]);
                gt[q] = in && k > thr;
                eq[q] = in && k == thr;
                ne += eq[q] ? 1u : 0u;
            }
            uint32_t etot;
            uint32_t erank = tie_run + ex_scan<NT>(ne, wsum, etot);        // ties before this thread's
            uint32_t na = 0;
            bool adm[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                adm[q] = gt[q] || (eq[q] && erank >= tie_from && erank < tie_to);
                erank += eq[q] ? 1u : 0u;
                na += adm[q] ? 1u : 0u;
            }
            uint32_t atot;
            uint32_t pos = base + ex_scan<NT>(na, wsum, atot);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (adm[q]) { oi[pos] = (uint32_t)(j0 + q); ov[pos] = v[q]; ++pos; }
            base += atot;
            tie_run += etot;
            if (sb == SUBS - 1 && t == 0) ws.tab[c * n + row] = make_uint2(cbase, base - cbase);
        }
        if (t == 0) {
            ws.thr[row] = thr;
            ws.krem[row] = krem;
            ws.rowcnt[row * RCS] = base;
            // the reason the fast path failed stays readable (flc_select_row_flags)
            ws.flags[row] = F_EXACT | (ws.flags[row] & (F_OVERFLOW | F_SHORT));
        }
        __syncthreads();
    }
}

template <bool VEC>
__global__ __launch_bounds__(EX_NT) void k_topk_exact_rows(RowSrc rows, int64_t n, int64_t r0, int64_t rn, int64_t d, int64_t K, SelWs ws) {
    __shared__ uint32_t h[HBINS];
    __shared__ uint32_t scratch[260];
    __shared__ uint32_t wsum[EX_NT / 64];
    for (int64_t row = r0 + blockIdx.x; row < r0 + rn; row += gridDim.x) {
        if (!(ws.flags[row] & (F_OVERFLOW | F_SHORT))) continue;       // row-uniform
        exact_row<VEC>(rows, n, row, d, K, ws, h, scratch, wsum);
    }
}

// The many-row candidate select with the exact fallback in the same workgroup: a row whose list
// overflowed in the filter, came up short, or whose K-th key the digits could not settle is
// selected exactly right here (exact_row with this workgroup's NT threads), so the group's
// select leaves every row final and no separate exact launch (a grid of 1024-thread workgroups
// that waited for whole CUs beside the next filter) follows it.
template <int NT, bool VEC>
__global__ __launch_bounds__(NT) void k_cand_select_x(RowSrc rows, int64_t n, int64_t r0, int64_t rn, int64_t d, int64_t K,
                                                      SelWs ws) {
    __shared__ uint32_t h[HBINS];
    __shared__ uint32_t scratch[260];
    __shared__ uint32_t wsum[NT / 64];
    __shared__ uint32_t failed;
    for (int64_t row = r0 + blockIdx.x; row < r0 + rn; row += gridDim.x) {
        cand_select_row<NT>(row, K, ws, h, scratch);
        __syncthreads();
        if (threadIdx.x == 0) failed = __atomic_load_n(&ws.flags[row], __ATOMIC_RELAXED) & (F_OVERFLOW | F_SHORT);
        __syncthreads();
        if (failed) exact_row<VEC, NT>(rows, n, row, d, K, ws, h, scratch, wsum);
        __syncthreads();
    }
}

// Exact path, ambiguous ties: per chunk count of key == thr, then the exclusive prefix over
// chunks (in index order) per row.  RowSrc without F_TIES get tieprefix = 0 (krem admits all ties).
__global__ __launch_bounds__(256) void k_tie_count(RowSrc rows, int64_t n, int64_t d, SelWs ws) {
    const int64_t C = nchunks(d);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t nrows = *ws.nwork;
    const int64_t bpr = (C + 3) / 4;
    for (int64_t it = blockIdx.x; it < nrows * bpr; it += gridDim.x) {
        const int64_t row = ws.worklist[it / bpr];
        const int64_t c = (it % bpr) * 4 + wv;
        if (c >= C) continue;
        uint32_t cnt = 0;
        if (ws.flags[row] & F_TIES) {
            const uint32_t T = ws.thr[row];
            const float* r = rows.row(row);
            const int64_t j1 = min(d, (c + 1) * (int64_t)CHUNK);
            for (int64_t j = c * CHUNK + lane; j < j1; j += 64) cnt += (mag_key(r[j]) == T) ? 1u : 0u;
            cnt = wave_sum(cnt);
        }
        if (lane == 0) ws.tieprefix[c * n + row] = cnt;
    }
}

// Exclusive prefix of the per-chunk tie counts, in chunk (= index) order, for the exact-path
// worklist rows.
__global__ __launch_bounds__(256) void k_tie_scan(int64_t n, int64_t d, SelWs ws) {
    constexpr bool EXACT = true;
    __shared__ uint32_t part[256];
    const int64_t C = nchunks(d);
    const int64_t nrows = EXACT ? (int64_t)(*ws.nwork) : n;
    const int t = threadIdx.x;
    const int64_t per = (C + 255) / 256;           // chunks per thread (contiguous)
    for (int64_t li = blockIdx.x; li < nrows; li += gridDim.x) {
        const int64_t row = EXACT ? (int64_t)ws.worklist[li] : li;
        if (!EXACT && (ws.flags[row] & (F_TIES | F_EXACT)) != F_TIES) continue;
        const int64_t c0 = t * per, c1 = min(C, c0 + per);
        uint32_t sum = 0;
        for (int64_t c = c0; c < c1; ++c) sum += ws.tieprefix[c * n + row];
        part[t] = sum;
        __syncthreads();
        for (int off = 1; off < 256; off <<= 1) {
            const uint32_t v = (t >= off) ? part[t - off] : 0u;
            __syncthreads();
            part[t] += v;
            __syncthreads();
        }
        uint32_t run = part[t] - sum;              // exclusive
        for (int64_t c = c0; c < c1; ++c) {
            const uint32_t v = ws.tieprefix[c * n + row];
            ws.tieprefix[c * n + row] = run;
            run += v;
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------
// RandK compat lists (indices given: the reference's numpy-stream draws)
// ------------------------------------------------------------------------------------------
// Chunk-bucketed RandK lists in two coalesced levels.
//   k_randk_coarse (one workgroup per row): the row's K indices copied once into the row's ent_val region;
//     LDS counts per superchunk (SB buckets of SPC chunks), LDS scan, then each index appended to
//     its superchunk's segment of ent_idx: SB write frontiers per row, which stay in L2.
//   k_randk_fine (one workgroup per (superchunk, row)): counting sort of the segment by chunk with
//     LDS counters (the segment is copied to ent_val first, scattered back inside the segment),
//     the (offset, count) table entries, then the gather (D/K) * x[j] in ascending chunk order.
constexpr int RK_T = 1024;
constexpr int RK_SB = 256;                   // superchunks per row (max)
constexpr int RK_TILE = 8192;                // indices per LDS multi-split tile (32 KB)

__host__ __device__ inline int64_t rk_spc(int64_t C) { return (C + RK_SB - 1) / RK_SB; }   // chunks per superchunk

template <class Emit>
__device__ inline void randk_walk(const flc_pattern& pat, int64_t row, int64_t K, int64_t ldi, int tid, Emit emit) {
    for (int64_t t = tid; t < K; t += RK_T) emit(t, (uint32_t)pat.d_randk_idx[row * ldi + t]);
}

// FINAL (one chunk per superchunk, C <= RK_SB): the superchunks are the chunks, so this kernel also
// writes the (offset, count) table and gathers the values; k_randk_fine is skipped.
template <bool FINAL>
__global__ __launch_bounds__(RK_T) void k_randk_coarse(RowSrc rows, int64_t n, int64_t d, int64_t K, flc_pattern pat,
                                                       int64_t ldi, float scale, SelWs ws) {
    __shared__ uint32_t cnt[RK_SB], tcnt[RK_SB], toff[RK_SB], gbase[RK_SB];
    __shared__ uint32_t tile[RK_TILE];
    const int64_t row = blockIdx.x;
    const int64_t C = nchunks(d), spc = rk_spc(C);
    const int tid = threadIdx.x;
    if (tid < RK_SB) cnt[tid] = 0;
    __syncthreads();
    uint32_t* jbuf = reinterpret_cast<uint32_t*>(ws.ent_val + row * ws.cap);
    randk_walk(pat, row, K, ldi, tid, [&](int64_t t, uint32_t j) {
        jbuf[t] = j;
        atomicAdd(&cnt[(j >> CHUNK_SHIFT) / spc], 1u);
    });
    __syncthreads();
    if (tid < 64) {                          // exclusive scan of the RK_SB counts: 4 per lane
        uint32_t v[RK_SB / 64], loc = 0;
#pragma unroll
        for (int q = 0; q < RK_SB / 64; ++q) { v[q] = cnt[tid * (RK_SB / 64) + q]; loc += v[q]; }
        uint32_t incl = loc;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = __shfl_up(incl, o, WAVE);
            if (tid >= o) incl += u;
        }
        uint32_t run = incl - loc;
#pragma unroll
        for (int q = 0; q < RK_SB / 64; ++q) {
            const int b = tid * (RK_SB / 64) + q;
            if (FINAL) {
                if (b < C) ws.tab[(int64_t)b * n + row] = make_uint2(run, v[q]);
            } else {
                ws.cursor[row * RK_SB + b] = run;         // segment offsets, read by k_randk_fine
            }
            cnt[b] = run;
            run += v[q];
        }
    }
    __syncthreads();
    // Append to the superchunk segments tile by tile: an LDS counting sort of RK_TILE indices, then
    // each bucket's run of the tile is written contiguously (a scattered 4-B store per index would
    // run at a small fraction of the store rate).  Thread tid only re-reads jbuf slots it wrote.
    uint32_t* oi = ws.ent_idx + row * ws.cap;
    constexpr int Q = RK_TILE / RK_T;
    for (int64_t t0 = 0; t0 < K; t0 += RK_TILE) {
        const int m = (int)min<int64_t>(RK_TILE, K - t0);
        if (tid < RK_SB) tcnt[tid] = 0;
        __syncthreads();
        uint32_t jj[Q], rnk[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int k = tid + q * RK_T;
            if (k < m) {
                jj[q] = jbuf[t0 + k];
                rnk[q] = atomicAdd(&tcnt[(jj[q] >> CHUNK_SHIFT) / spc], 1u);
            }
        }
        __syncthreads();
        if (tid < 64) {
            uint32_t v[RK_SB / 64], loc = 0;
#pragma unroll
            for (int q = 0; q < RK_SB / 64; ++q) { v[q] = tcnt[tid * (RK_SB / 64) + q]; loc += v[q]; }
            uint32_t incl = loc;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t u = __shfl_up(incl, o, WAVE);
                if (tid >= o) incl += u;
            }
            uint32_t run = incl - loc;
#pragma unroll
            for (int q = 0; q < RK_SB / 64; ++q) {
                const int b = tid * (RK_SB / 64) + q;
                toff[b] = run;
                gbase[b] = cnt[b];
                cnt[b] += v[q];
                run += v[q];
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int k = tid + q * RK_T;
            if (k < m) tile[toff[(jj[q] >> CHUNK_SHIFT) / spc] + rnk[q]] = jj[q];
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int k = tid + q * RK_T;
            if (k < m) {
                const uint32_t j = tile[k];
                const uint32_t b = (j >> CHUNK_SHIFT) / spc;
                oi[gbase[b] + (uint32_t)k - toff[b]] = j;
            }
        }
        __syncthreads();
    }
    if (tid == 0) {
        ws.thr[row] = 0;
        ws.flags[row] = F_EXACT;
        ws.rowcnt[row * RCS] = (uint32_t)K;
    }
    if (FINAL) {
        __syncthreads();                                  // block-scope visibility of the idx writes
        const float* r = rows.row(row);
        float* val = ws.ent_val + row * ws.cap;
        for (int64_t t = tid; t < K; t += RK_T) val[t] = scale * r[oi[t]];   // (D/K) * x[S] in fp32
    }
}

// Segments up to RK_FT entries (the device sampler's ~K / RK_SB, far above any binomial tail) are
// sorted in LDS and written back, with the values, in one coalesced sweep; a larger segment (an
// arbitrary compat index list) takes the slower in-memory counting sort.
constexpr int RK_FT = 8192, RK_FTHR = 512;
__global__ __launch_bounds__(RK_FTHR) void k_randk_fine(RowSrc rows, int64_t n, int64_t d, int64_t K, float scale,
                                                        SelWs ws) {
    extern __shared__ uint32_t fc[];                       // [spc] counts, then offsets / cursors
    __shared__ uint32_t wsum[RK_FTHR / 64];
    __shared__ uint32_t tile[RK_FT];
    const int64_t row = blockIdx.y, b = blockIdx.x;
    const int64_t C = nchunks(d), spc = rk_spc(C);
    const int64_t cb0 = b * spc, cb1 = min(C, cb0 + spc);
    const int tid = threadIdx.x;
    if (cb0 >= C) return;
    const uint32_t s0 = ws.cursor[row * RK_SB + b];
    const uint32_t s1 = (b + 1 < RK_SB) ? ws.cursor[row * RK_SB + b + 1] : (uint32_t)K;
    const int64_t nc = cb1 - cb0;
    const bool in_lds = s1 - s0 <= (uint32_t)RK_FT;
    for (int64_t c = tid; c < nc; c += RK_FTHR) fc[c] = 0;
    __syncthreads();
    uint32_t* idx = ws.ent_idx + row * ws.cap;
    uint32_t* tmp = reinterpret_cast<uint32_t*>(ws.ent_val + row * ws.cap);
    constexpr int Q = RK_FT / RK_FTHR;
    uint32_t jj[Q], rnk[Q];
    if (in_lds) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const uint32_t t = s0 + tid + q * RK_FTHR;
            if (t < s1) {
                jj[q] = idx[t];
                rnk[q] = atomicAdd(&fc[(jj[q] >> CHUNK_SHIFT) - cb0], 1u);
            }
        }
    } else {
        for (uint32_t t = s0 + tid; t < s1; t += RK_FTHR) {
            const uint32_t j = idx[t];
            tmp[t] = j;
            atomicAdd(&fc[(j >> CHUNK_SHIFT) - cb0], 1u);
        }
    }
    __syncthreads();
    // exclusive scan of nc counters: thread t owns a contiguous block
    const int64_t per = (nc + RK_FTHR - 1) / RK_FTHR;
    const int64_t q0 = min<int64_t>(nc, tid * per), q1 = min<int64_t>(nc, q0 + per);
    uint32_t loc = 0;
    for (int64_t c = q0; c < q1; ++c) loc += fc[c];
    uint32_t incl = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(incl, o, WAVE);
        if ((tid & 63) >= o) incl += u;
    }
    if ((tid & 63) == 63) wsum[tid >> 6] = incl;
    __syncthreads();
    uint32_t run = incl - loc;
    for (int w = 0; w < (tid >> 6); ++w) run += wsum[w];
    for (int64_t c = q0; c < q1; ++c) {
        const uint32_t v = fc[c];
        ws.tab[(cb0 + c) * n + row] = make_uint2(s0 + run, v);
        fc[c] = run;                                        // segment-relative offset
        run += v;
    }
    __syncthreads();
    const float* r = rows.row(row);
    float* val = ws.ent_val + row * ws.cap;
    if (in_lds) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const uint32_t t = s0 + tid + q * RK_FTHR;
            if (t < s1) tile[fc[(jj[q] >> CHUNK_SHIFT) - cb0] + rnk[q]] = jj[q];
        }
        __syncthreads();
        for (uint32_t k = tid; k < s1 - s0; k += RK_FTHR) {
            const uint32_t j = tile[k];
            idx[s0 + k] = j;
            val[s0 + k] = scale * r[j];                     // (D/K) * x[S] in fp32, ascending columns
        }
        return;
    }
    for (uint32_t t = s0 + tid; t < s1; t += RK_FTHR) {
        const uint32_t j = tmp[t];
        idx[s0 + atomicAdd(&fc[(j >> CHUNK_SHIFT) - cb0], 1u)] = j;
    }
    __syncthreads();                                        // block-scope visibility of the idx writes
    for (uint32_t t = s0 + tid; t < s1; t += RK_FTHR) val[t] = scale * r[idx[t]];
}

// ------------------------------------------------------------------------------------------
// Chunk-owner accumulation.  One wave per chunk, fp32 tile in LDS; rows folded in order.
// ASSIGN (single row, no weights): out = tile with the entry values stored, not added
// (keeps -0.0 like torch's out[ind] = x[ind]).
// ------------------------------------------------------------------------------------------
// Admission per entry: exact-path rows (F_EXACT) hold exactly their admitted entries; fast-path
// rows admit key > thr, and key == thr either all (no F_TIES) or up to the row's tie cut (the
// largest index admitted among the ties, k_cand_select).
//
// One wave owns one chunk: a 4096-float LDS tile into which the rows are folded in row order
// (bit-exact sequential sum; within a row the entries' columns are distinct).  The walk over the
// N rows is a software pipeline: the per-row state (tab entry, thr, cut, mode, weight) of 64 rows
// is fetched one batch ahead with lane = row, and the entry lists of the next AP rows are in
// flight while a row is folded (a ring of AP register slots, 2 x 64 entries per row), so the
// wave never waits on a dependent tab -> entries round trip.
// ------------------------------------------------------------------------------------------
#ifndef FLC_CA_PROBE
#define FLC_CA_PROBE 0               // A/B cost probe of k_chunk_accum (outputs NOT valid): 1 no tile update
#endif
#ifndef FLC_CA_AP1
#define FLC_CA_AP1 4                 // one-wave fold workgroups: rows in flight (<= 113 VGPRs: beside the TopK filter's 3 waves per SIMD)
#endif
#ifndef FLC_CA_WPB1
#define FLC_CA_WPB1 0                // k_chunk_accum over whole chunks: one-wave workgroups
#endif
#ifndef FLC_CA_AP
#define FLC_CA_AP 8
#endif
constexpr int AP = FLC_CA_AP;              // rows of entry lists in flight

struct RowMeta {
    uint2 te;          // (offset, count) of the row's list in this chunk
    uint32_t thr, cut, mode;   // cut: tie_pref of the row's tie cut (0 admits every tie)
    float w;
};

__device__ inline RowMeta load_meta(const SelWs& ws, int64_t c, int64_t n, int64_t r, const float* w, int64_t rend = -1) {
    RowMeta m;
    m.te = make_uint2(0, 0);
    m.thr = 0; m.cut = 0u; m.mode = 0; m.w = 1.f;
    if (r < (rend < 0 ? n : rend)) {
        m.te = ws.tab[c * n + r];
        m.thr = ws.thr[r];
        const uint32_t f = ws.flags[r];
        m.mode = (f & F_EXACT) ? 2u : ((f & F_TIES) ? 1u : 0u);
        if (m.mode == 1u) m.cut = tie_pref(ws.tiecut[r], ws.tie_hi);
        if (m.mode == 2u) m.thr = 0u;          // exact list: every entry admitted (key >= 0, cut ~0)
        if (w) m.w = w[r];
    }
    return m;
}


// Sign of zero.  The reference adds every client's DENSE row, so a column a row did not keep
// receives the term w_i * (+0) (-0 when w_i's sign bit is set).  The fold skips those terms and
// starts its tile at -0 (the additive identity), which gives the same bits for every nonzero
// result.  A sum is -0 only if every term was -0: the tile ends at -0 exactly when every KEPT
// term was -0 (or none was kept), and the reference's sum is then -0 iff, in addition, every row
// that did not keep the column has a negative-signed weight.  Those columns are resolved here:
// for each row with a positive-signed weight (stopping once no candidate is left) the -0
// columns it does not keep turn +0.  Untouched columns die at the first such row, so this costs
// one extra list walk for chunks that have them and nothing for the others.
template <int TS>
__device__ void resolve_neg_zero(float* tl, uint32_t* rm, const SelWs& ws, int64_t c, int64_t n, uint32_t cbase,
                                 int64_t len, const float* w, int lane) {
    constexpr int NW = TS / 32;                        // mask words (32 columns each)
    constexpr int WL = (NW + 63) / 64;                 // mask words per lane (word k = lane + 64 j)
    bool any = false;
    for (int k = 0; k < TS / 64; ++k) {
        const int64_t i = (int64_t)k * 64 + lane;
        const uint64_t b = __ballot(i < len && __float_as_uint(tl[i]) == 0x80000000u);
        if (lane == 0) { rm[2 * k] = (uint32_t)b; rm[2 * k + 1] = (uint32_t)(b >> 32); }
        any |= b != 0ull;
    }
    if (!any) return;
    uint32_t z0[WL], zc[WL];
#pragma unroll
    for (int j = 0; j < WL; ++j) {
        const int k = lane + 64 * j;
        z0[j] = k < NW ? rm[k] : 0u;
        zc[j] = z0[j];
    }
    for (int64_t r = 0; r < n; ++r) {
        if (w && (__float_as_uint(w[r]) >> 31)) continue;      // its skipped term is -0: no constraint
#pragma unroll
        for (int j = 0; j < WL; ++j) if (lane + 64 * j < NW) rm[lane + 64 * j] = 0u;
        const RowMeta m = load_meta(ws, c, n, r, w);
        const uint32_t mode = m.mode, T = m.thr, cut = m.cut;
        for (uint32_t e = (uint32_t)lane; e < m.te.y; e += 64) {
            const uint32_t ix = ws.ent_idx[r * ws.cap + m.te.x + e];
            const uint32_t key = mag_key(ws.ent_val[r * ws.cap + m.te.x + e]);
            const uint32_t loc = ix - cbase;
            if (loc < (uint32_t)TS && (mode == 2u || key > T || (key == T && tie_pref(ix, ws.tie_hi) >= cut)))
                atomicOr(&rm[loc >> 5], 1u << (loc & 31));
        }
        bool left = false;
#pragma unroll
        for (int j = 0; j < WL; ++j) {
            if (lane + 64 * j < NW) zc[j] &= rm[lane + 64 * j];
            left |= zc[j] != 0u;
        }
        if (__ballot(left) == 0ull) break;
    }
#pragma unroll
    for (int j = 0; j < WL; ++j) {
        uint32_t dead = z0[j] & ~zc[j];
        while (dead) {
            const int b = __builtin_ctz(dead);
            dead &= dead - 1u;
            tl[(lane + 64 * j) * 32 + b] = 0.f;
        }
    }
}

// resolve_neg_zero for one-wave workgroups whose LDS holds only the tile: the -0 column masks
// live in registers (word k of the tile's TS / 32 in lane k % 64), a row's kept columns are OR-ed
// into the job's global scratch `rm` (TS / 32 words) and read back at L2 (atomic reads: no stale
// L1 line).  Same rule, same bits; it runs once per job and usually stops after one row.
template <int TS>
__device__ void resolve_neg_zero_g(float* tl, uint32_t* rm, const SelWs& ws, int64_t c, int64_t n, uint32_t cbase,
                                   int64_t len, const float* w, int lane) {
    constexpr int NW = TS / 32;                        // mask words (32 columns each)
    constexpr int WL = (NW + 63) / 64;                 // mask words per lane (word k = lane + 64 j)
    uint32_t z0[WL], zc[WL];
#pragma unroll
    for (int j = 0; j < WL; ++j) z0[j] = 0u;
    bool any = false;
#pragma unroll 4
    for (int k = 0; k < TS / 64; ++k) {
        const int64_t i = (int64_t)k * 64 + lane;
        const uint64_t b = __ballot(i < len && __float_as_uint(tl[i]) == 0x80000000u);
        const int w0 = 2 * k, w1 = 2 * k + 1;          // words of columns 64 k .. 64 k + 63
#pragma unroll
        for (int j = 0; j < WL; ++j) {
            if (lane == (w0 & 63) && (w0 >> 6) == j) z0[j] = (uint32_t)b;
            if (lane == (w1 & 63) && (w1 >> 6) == j) z0[j] = (uint32_t)(b >> 32);
        }
        any |= b != 0ull;
    }
    if (!any) return;
#pragma unroll
    for (int j = 0; j < WL; ++j) zc[j] = z0[j];
    for (int64_t r = 0; r < n; ++r) {
        if (w && (__float_as_uint(w[r]) >> 31)) continue;      // its skipped term is -0: no constraint
#pragma unroll
        for (int j = 0; j < WL; ++j) if (lane + 64 * j < NW) rm[lane + 64 * j] = 0u;
        __threadfence_block();
        const RowMeta m = load_meta(ws, c, n, r, w);
        const uint32_t mode = m.mode, T = m.thr, cut = m.cut;
        for (uint32_t e = (uint32_t)lane; e < m.te.y; e += 64) {
            const uint32_t ix = ws.ent_idx[r * ws.cap + m.te.x + e];
            const uint32_t key = mag_key(ws.ent_val[r * ws.cap + m.te.x + e]);
            const uint32_t loc = ix - cbase;
            if (loc < (uint32_t)TS && (mode == 2u || key > T || (key == T && tie_pref(ix, ws.tie_hi) >= cut)))
                atomicOr(&rm[loc >> 5], 1u << (loc & 31));
        }
        __threadfence_block();
        bool left = false;
#pragma unroll
        for (int j = 0; j < WL; ++j) {
            if (lane + 64 * j < NW) zc[j] &= atomicOr(&rm[lane + 64 * j], 0u);
            left |= zc[j] != 0u;
        }
        if (__ballot(left) == 0ull) break;
    }
#pragma unroll
    for (int j = 0; j < WL; ++j) {
        uint32_t dead = z0[j] & ~zc[j];
        while (dead) {
            const int b = __builtin_ctz(dead);
            dead &= dead - 1u;
            tl[(lane + 64 * j) * 32 + b] = 0.f;
        }
    }
}

// TS < CHUNK: a wave owns TS columns of a chunk (CHUNK / TS waves read the same lists and each
// folds its part): a smaller LDS tile per wave, so more waves per CU hide the list latency.
// WPB = 1 (whole chunks): one-wave workgroups holding only their 16 KB tile, so ten fit a CU's
// 160 KB and every chunk of a 10 M row (2442) has its wave resident at once — with 4-wave blocks
// (67.5 KB with the masks) two fit a CU, 2048 chunk waves ran and the last 394 formed a second
// round of the same length.
// Row groups: rows [r0, rend) only; `first` starts the tiles at -0, else from ws.part (the previous
// group's tiles); `last` resolves the -0 columns over ALL n rows and writes out = sums / wt, else
// the tiles go back to ws.part.  (r0 = 0, rend = n, first = last = 1: one fold of every row.)
template <bool ASSIGN, int TS, bool W, int WPB, int AP = AP>
__device__ __forceinline__ void chunk_accum_body(int64_t n, int64_t d, SelWs ws, const float* __restrict__ w, float wt,
                                                 float* __restrict__ out, int64_t r0, int64_t rend, int first, int last,
                                                 float (*tile)[TS], uint32_t (*zmask)[WPB == 1 ? 1 : TS / 32]) {
    if (rend < 0) rend = n;
    constexpr int PARTS = CHUNK / TS;
    const int lane = threadIdx.x & 63;
    const int wv = WPB == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t C = nchunks(d);
    float* tl = tile[wv];
    const int64_t nb = (rend - r0 + 63) / 64;          // row batches
    for (int64_t t = (int64_t)blockIdx.x * WPB + wv; t < C * PARTS; t += (int64_t)gridDim.x * WPB) {
        const int64_t c = t / PARTS;
        const uint32_t cbase = (uint32_t)(c * CHUNK + (t % PARTS) * TS);
        // ASSIGN (compressVector: out = zeros, out[kept] = x) stores into +0; the fold adds into -0
        if (FLC_TILE_V4 && !ASSIGN && !first && (int64_t)cbase + TS <= d) {
            // the carried tile with its loads in flight 8 float4 at a time (the loop of load -> LDS
            // write pairs below waits one memory latency per 64 columns: 64 per 4096-column tile)
            const float4* p4 = reinterpret_cast<const float4*>(ws.part + cbase);
#pragma unroll
            for (int k0 = 0; k0 < TS / 256; k0 += 8) {
                float4 v[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = k0 + k < TS / 256 ? p4[(k0 + k) * 64 + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if (k0 + k < TS / 256) reinterpret_cast<float4*>(tl)[(k0 + k) * 64 + lane] = v[k];
            }
        } else {
            for (int i = lane; i < TS; i += 64)
                tl[i] = ASSIGN ? 0.f : (first || (int64_t)cbase + i >= d ? -0.f : ws.part[cbase + i]);
        }
        RowMeta cur = load_meta(ws, c, n, r0 + lane, w, rend), nxt;
        // ring of AP rows' entries (the first 128 of each list; range-checked buffer loads, lanes
        // past the list end get index ~0 = no column)
        uint32_t ri[AP][2];
        float rv[AP][2];
        auto fetch = [&](const RowMeta& m, int q, int64_t row, int slot) {
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
        // admission (key > T, or key == T and tie_pref(ix) >= tie_pref(cut); load_meta folds the
        // exact mode into T = 0, cut 0) as ONE 64-bit compare: (key, tie_pref(ix)) >= (T, cut)
        const uint32_t txm = ws.tie_hi ? 0u : 0xFFFFFFFFu;   // tie_pref(ix) = ix ^ txm
        auto fold = [&](uint32_t ix, float vv, uint32_t T, uint32_t cut, uint32_t mode, float wi) {
            (void)mode;
            const uint32_t loc = ix - cbase;                   // ~0 index / other part: loc >= TS
            const uint64_t a = ((uint64_t)mag_key(vv) << 32) | (uint64_t)(ix ^ txm);
            const uint64_t b = ((uint64_t)T << 32) | (uint64_t)cut;
            if (FLC_CA_PROBE == 1) {                          // cost probe: no tile update
                if (loc < (uint32_t)TS && a >= b && vv == 1.2345f) tl[0] = vv;
                return;
            }
            if (loc < (uint32_t)TS && a >= b) {
                if (ASSIGN) tl[loc] = vv;
                else tl[loc] = W ? tl[loc] + wi * vv : tl[loc] + vv;
            }
        };
#pragma unroll
        for (int q = 0; q < AP; ++q) fetch(cur, q, r0 + q, q);
        for (int64_t b = 0; b < nb; ++b) {
            const int64_t i0 = r0 + b * 64;
            nxt = load_meta(ws, c, n, i0 + 64 + lane, w, rend);   // next batch's state, one batch ahead
            if (__builtin_expect(__ballot(cur.te.y > 128u) == 0ull, 1)) {
                // every list of the batch fits the ring slots: straight-line pipeline
#pragma unroll
                for (int q = 0; q < 64; ++q) {
                    const int slot = q % AP;
                    const uint32_t T = __builtin_amdgcn_readlane(cur.thr, q);
                    const uint32_t cut = __builtin_amdgcn_readlane(cur.cut, q);
                    const uint32_t mode = 0u;
                    const float wi = W ? __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(cur.w), q)) : 1.f;
                    fold(ri[slot][0], rv[slot][0], T, cut, mode, wi);
                    // the second slot holds entries only when the list is longer than 64
                    if (__builtin_amdgcn_readlane(cur.te.y, q) > 64u) fold(ri[slot][1], rv[slot][1], T, cut, mode, wi);
                    if (q + AP < 64) fetch(cur, q + AP, i0 + q + AP, slot);
                    else fetch(nxt, q + AP - 64, i0 + q + AP, slot);   // past n: empty lists
                }
            } else {
                // some list is longer than 128 entries: the same walk with the tails folded in place
                for (int q = 0; q < 64; ++q) {
                    const int slot = q % AP;
                    const uint32_t T = __shfl(cur.thr, q, WAVE), cut = __shfl(cur.cut, q, WAVE);
                    const uint32_t mode = __shfl(cur.mode, q, WAVE), cnt = __shfl(cur.te.y, q, WAVE);
                    const uint32_t off = __shfl(cur.te.x, q, WAVE);
                    const float wi = W ? __shfl(cur.w, q, WAVE) : 1.f;
                    uint32_t i_0 = 0, i_1 = 0;
                    float v_0 = 0.f, v_1 = 0.f;
#pragma unroll
                    for (int z = 0; z < AP; ++z)
                        if (z == slot) { i_0 = ri[z][0]; i_1 = ri[z][1]; v_0 = rv[z][0]; v_1 = rv[z][1]; }
                    fold(i_0, v_0, T, cut, mode, wi);
                    fold(i_1, v_1, T, cut, mode, wi);
                    const int64_t row = i0 + q;
                    for (uint32_t e = 128u + lane; e < cnt; e += 64)
                        fold(ws.ent_idx[row * ws.cap + off + e], ws.ent_val[row * ws.cap + off + e], T, cut, mode, wi);
                    // refill the slot (same contract as the straight-line path)
                    const RowMeta& m = (q + AP < 64) ? cur : nxt;
                    const int qq = (q + AP) & 63;
                    const uint32_t offn = __shfl(m.te.x, qq, WAVE), cntn = __shfl(m.te.y, qq, WAVE);
                    const int64_t rown = i0 + q + AP;
                    uint32_t xi[2];
                    float xv[2];
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const uint32_t e = (uint32_t)lane + 64u * h;
                        xi[h] = e < cntn ? ws.ent_idx[rown * ws.cap + offn + e] : 0xFFFFFFFFu;
                        xv[h] = e < cntn ? ws.ent_val[rown * ws.cap + offn + e] : 0.f;
                    }
#pragma unroll
                    for (int z = 0; z < AP; ++z)
                        if (z == slot) { ri[z][0] = xi[0]; ri[z][1] = xi[1]; rv[z][0] = xv[0]; rv[z][1] = xv[1]; }
                }
            }
            cur = nxt;
        }
        const int64_t len = min((int64_t)TS, d - (int64_t)cbase);
        if (!last) {                                   // row groups: the tiles carry on to the next group
            for (int64_t i = lane; i < len; i += 64) ws.part[cbase + i] = tl[i];
            continue;
        }
        if (!ASSIGN) {
            if (WPB == 1) resolve_neg_zero_g<TS>(tl, ws.zm + t * (TS / 32), ws, c, n, cbase, len, w, lane);
            else resolve_neg_zero<TS>(tl, zmask[wv], ws, c, n, cbase, len, w, lane);
        }
        for (int64_t i = lane; i < len; i += 64) out[cbase + i] = ASSIGN ? tl[i] : tl[i] / wt;
    }
}

template <bool ASSIGN, int TS = CHUNK, bool W = true>
__global__ __launch_bounds__(256) void k_chunk_accum(int64_t n, int64_t d, SelWs ws, const float* __restrict__ w, float wt,
                                                     float* __restrict__ out, int64_t r0 = 0, int64_t rend = -1,
                                                     int first = 1, int last = 1) {
    __shared__ __attribute__((aligned(16))) float tile[4][TS];
    __shared__ uint32_t zmask[4][TS / 32];
    chunk_accum_body<ASSIGN, TS, W, 4>(n, d, ws, w, wt, out, r0, rend, first, last, tile, zmask);
}

// one-wave workgroups holding only their tile (16 KB) and at most FLC_CA_VGPR1 VGPRs: they fit in
// what the TopK filter's waves leave free on a CU (row-group folds under the next group's filter)
// (the tile is dynamic LDS, CHUNK floats given at launch: with a static 16 KB array the compiler
// takes LDS as the occupancy limit and ignores the waves-per-EU request)
template <bool W>
__global__ __launch_bounds__(64) void k_chunk_accum1(
        int64_t n, int64_t d, SelWs ws, const float* __restrict__ w, float wt, float* __restrict__ out, int64_t r0,
        int64_t rend, int first, int last) {
    extern __shared__ __attribute__((aligned(16))) float dyn_tile[];
    chunk_accum_body<false, CHUNK, W, 1, FLC_CA_AP1>(n, d, ws, w, wt, out, r0, rend, first, last,
                                         reinterpret_cast<float (*)[CHUNK]>(dyn_tile), nullptr);
}

// ------------------------------------------------------------------------------------------
// RandK device mode (randk_tree.hpp): no index lists.
//   k_randk_counts : one workgroup per row walks the hypergeometric tree level by level (ping-pong
//                    level arrays in the workspace) -> cnt[c][row] = the row's members in chunk c,
//                    and the row's client key
//   k_randk_fold   : one wave per chunk (or 1/2, 1/4 of its columns when the rows are short) folds
//                    the rows in order into an fp32 LDS tile: row q's members of the chunk are the
//                    first cnt[c][q] images of the chunk permutation (lane t -> offset P(t)), their
//                    values (D/K) * x_q[j] gathered with range-checked buffer loads (AP rows in
//                    flight), added as w_q * v — the sequential fold of the dense compressVector
//                    outputs, bit for bit (a row's members are distinct)
// ------------------------------------------------------------------------------------------
struct RkdWs {
    uint32_t* cnt;     // [C][N]
    uint64_t* ckey;    // [N]
};

// Chunk counts of the device sampler (randk_tree.hpp): each workgroup takes one row and a range of
// RKC_BINS chunks, evaluates Pi(t) for all t < K with a persistent cycle walk (every lane does
// useful work each trip) and histograms the chunk ids in LDS (16-bit bins: a chunk holds <= 4096).
constexpr int RKC_NT = 1024;
constexpr int64_t RKC_BINS = 32768;

// the client keys of the device sampler (k_randk_counts writes them beside the counts)
__global__ __launch_bounds__(256) void k_randk_ckeys(int64_t n, uint64_t seed, int64_t client0, uint64_t* __restrict__ ckey) {
    const int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (row < n) ckey[row] = client_key(seed, client0 + row);
}

__global__ __launch_bounds__(RKC_NT) void k_randk_counts(int64_t n, int64_t d, int64_t K, uint64_t seed, int64_t client0,
                                                         RkdWs ws) {
    __shared__ uint32_t bins[RKC_BINS / 2];
    const int64_t row = blockIdx.y;
    const int tid = threadIdx.x;
    const int64_t C = nchunks(d);
    const int64_t c0 = (int64_t)blockIdx.x * RKC_BINS, nc = min(C, c0 + RKC_BINS) - c0;
    const uint64_t ck = client_key(seed, client0 + row);
    for (int64_t i = tid; i < (nc + 1) / 2; i += RKC_NT) bins[i] = 0;
    __syncthreads();
    const rktree::RowPerm P(ck, (uint64_t)d);
    int64_t t = tid;
    bool live = t < K;
    uint64_t x = (uint64_t)t;
    while (__ballot(live) != 0ull) {
        const uint64_t v = P.once(x);
        if (live) {
            if (v < (uint64_t)d) {
                const int64_t c = (int64_t)(v >> CHUNK_SHIFT) - c0;
                if ((uint64_t)c < (uint64_t)nc) atomicAdd(&bins[c >> 1], 1u << (16 * (c & 1)));
                t += RKC_NT;
                live = t < K;
                x = (uint64_t)t;
            } else {
                x = v;
            }
        }
    }
    __syncthreads();
    if (blockIdx.x == 0 && tid == 0) ws.ckey[row] = ck;
    for (int64_t c = tid; c < nc; c += RKC_NT) ws.cnt[(c0 + c) * n + row] = (bins[c >> 1] >> (16 * (c & 1))) & 0xFFFFu;
}

// lists view of the counts (the short-row path): tab[c][row] = (offset, count) with the members
// laid out chunk by chunk, and the F_EXACT row state (every listed entry is kept)
__global__ __launch_bounds__(256) void k_randk_tab(int64_t n, int64_t d, int64_t K, const uint32_t* __restrict__ cnt,
                                                   SelWs ls) {
    __shared__ uint32_t part[256];
    const int64_t row = blockIdx.x;
    const int tid = threadIdx.x;
    const int64_t C = nchunks(d), per = (C + 255) / 256;
    const int64_t c0 = min(C, tid * per), c1 = min(C, c0 + per);
    uint32_t loc = 0;
    for (int64_t c = c0; c < c1; ++c) loc += cnt[c * n + row];
    part[tid] = loc;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
        const uint32_t v = tid >= off ? part[tid - off] : 0u;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    uint32_t run = part[tid] - loc;
    for (int64_t c = c0; c < c1; ++c) {
        const uint32_t m = cnt[c * n + row];
        ls.tab[c * n + row] = make_uint2(run, m);
        run += m;
    }
    if (tid == 0) {
        ls.thr[row] = 0;
        ls.flags[row] = F_EXACT;
        ls.rowcnt[row * RCS] = (uint32_t)K;
    }
}

// Row-major member generation + gather: each wave takes RKG_CPW consecutive chunks of one row,
// lane t < m_c writes member t of chunk c (its global index and (D/K) x[j]) at the row's list
// position tab[c][row].x + t — the lists k_chunk_accum folds.  The gathers of a wave stay inside one
// row's 16 KB windows, chunk after chunk (page- and DRAM-row-local, like the compat path's
// k_randk_fine); the RKG_CPW chunks' loads are issued before any store.
constexpr int RKG_CPW = 4;
__global__ __launch_bounds__(256) void k_randk_gen(RowSrc rows, int64_t n, int64_t d, const uint64_t* __restrict__ ckey,
                                                   float scale, SelWs ws) {
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t C = nchunks(d);
    for (int64_t row = blockIdx.y; row < n; row += gridDim.y) {
        const uint64_t k = ckey[row];
        const float* r = rows.row_s(row);
        uint32_t* oi = ws.ent_idx + row * ws.cap;
        float* ov = ws.ent_val + row * ws.cap;
        for (int64_t c0 = ((int64_t)blockIdx.x * 4 + wv) * RKG_CPW; c0 < C; c0 += (int64_t)gridDim.x * 4 * RKG_CPW) {
            uint2 te[RKG_CPW];
            uint32_t col[RKG_CPW];
            float v[RKG_CPW];
#pragma unroll
            for (int q = 0; q < RKG_CPW; ++q) {
                const int64_t c = c0 + q;
                te[q] = c < C ? ws.tab[c * n + row] : make_uint2(0u, 0u);
                const uint32_t clen = (uint32_t)min((int64_t)CHUNK, d - c * CHUNK);
                const rktree::ChunkPerm P(k, c, clen);
                col[q] = (uint32_t)lane < te[q].y ? P((uint32_t)lane) : 0u;
                v[q] = (uint32_t)lane < te[q].y ? r[c * CHUNK + col[q]] : 0.f;
            }
#pragma unroll
            for (int q = 0; q < RKG_CPW; ++q) {
                const int64_t c = c0 + q;
                if ((uint32_t)lane < te[q].y) {
                    oi[te[q].x + lane] = (uint32_t)(c * CHUNK + col[q]);
                    ov[te[q].x + lane] = scale * v[q];
                }
                if (te[q].y > 64u) {                      // a chunk with more than 64 members
                    const uint32_t clen = (uint32_t)min((int64_t)CHUNK, d - c * CHUNK);
                    const rktree::ChunkPerm P(k, c, clen);
                    for (uint32_t t = 64u + lane; t < te[q].y; t += 64) {
                        const uint32_t cc = P(t);
                        oi[te[q].x + t] = (uint32_t)(c * CHUNK + cc);
                        ov[te[q].x + t] = scale * r[c * CHUNK + cc];
                    }
                }
            }
        }
    }
}

__device__ inline uint64_t join64(uint32_t hi, uint32_t lo) { return ((uint64_t)hi << 32) | (uint64_t)lo; }

struct RkMeta {            // lane = row of a 64-row batch
    uint32_t m;            // members of this chunk
    uint32_t klo, khi;     // client key
    uint32_t plo, phi;     // row pointer
    float w;
};

__device__ inline RkMeta rk_meta(RowSrc rows, const uint32_t* cnt, const uint64_t* ckey, const float* w, int64_t c,
                                 int64_t n, int64_t r, uint32_t clen) {
    RkMeta m{0u, 0u, 0u, 0u, 0u, 1.f};
    if (r < n) {
        m.m = min(cnt[c * n + r], clen);                 // <= clen by construction; never index past it
        const uint64_t k = ckey[r];
        m.klo = (uint32_t)k;
        m.khi = (uint32_t)(k >> 32);
        const uintptr_t p = (uintptr_t)rows.row(r);
        m.plo = (uint32_t)p;
        m.phi = (uint32_t)((uint64_t)p >> 32);
        if (w) m.w = w[r];
    }
    return m;
}

// -0 columns after the fold (every kept term was -0, or no row kept the column): the reference's
// sum is -0 only if every row's term is -0, and a row that did not keep the column adds w * (+0)
// (resolve_neg_zero above, the same rule).  Walk the rows with a positive-signed weight, regenerate
// their members of this part, and turn +0 every -0 column some such row does not keep; stops as
// soon as no candidate is left (normally after the first row).
template <int TS>
__device__ void rk_resolve_neg_zero(float* tl, uint32_t* rm, const uint32_t* cnt, const uint64_t* ckey, int64_t c,
                                    int64_t n, uint32_t pbase, uint32_t clen, int64_t len, const float* w, int lane) {
    constexpr int NW = TS / 32;
    constexpr int WL = (NW + 63) / 64;
    bool any = false;
    for (int k = 0; k < TS / 64; ++k) {
        const int64_t i = (int64_t)k * 64 + lane;
        const uint64_t b = __ballot(i < len && __float_as_uint(tl[i]) == 0x80000000u);
        if (lane == 0) { rm[2 * k] = (uint32_t)b; rm[2 * k + 1] = (uint32_t)(b >> 32); }
        any |= b != 0ull;
    }
    if (!any) return;
    uint32_t z0[WL], zc[WL];
#pragma unroll
    for (int j = 0; j < WL; ++j) {
        const int k = lane + 64 * j;
        z0[j] = k < NW ? rm[k] : 0u;
        zc[j] = z0[j];
    }
    for (int64_t r = 0; r < n; ++r) {
        if (w && (__float_as_uint(w[r]) >> 31)) continue;
#pragma unroll
        for (int j = 0; j < WL; ++j) if (lane + 64 * j < NW) rm[lane + 64 * j] = 0u;
        const uint32_t m = min(cnt[c * n + r], clen);
        const rktree::ChunkPerm P(ckey[r], c, clen);
        for (uint32_t t = (uint32_t)lane; t < m; t += 64) {
            const uint32_t loc = P(t) - pbase;
            if (loc < (uint32_t)TS) atomicOr(&rm[loc >> 5], 1u << (loc & 31));
        }
        bool left = false;
#pragma unroll
        for (int j = 0; j < WL; ++j) {
            if (lane + 64 * j < NW) zc[j] &= rm[lane + 64 * j];
            left |= zc[j] != 0u;
        }
        if (__ballot(left) == 0ull) break;
    }
#pragma unroll
    for (int j = 0; j < WL; ++j) {
        uint32_t dead = z0[j] & ~zc[j];
        while (dead) {
            const int b = __builtin_ctz(dead);
            dead &= dead - 1u;
            tl[(lane + 64 * j) * 32 + b] = 0.f;
        }
    }
}

#ifndef FLC_RK_AP
#define FLC_RK_AP 8
#endif
constexpr int RK_AP = FLC_RK_AP;
template <int TS>
__global__ __launch_bounds__(256) void k_randk_fold(RowSrc rows, int64_t n, int64_t d, const uint32_t* __restrict__ cnt,
                                                    const uint64_t* __restrict__ ckey, float scale,
                                                    const float* __restrict__ w, float wt, float* __restrict__ out) {
    constexpr int PARTS = CHUNK / TS;
    constexpr uint32_t NOCOL = 0xFFFFu;                    // past the chunk: the buffer load returns 0
    __shared__ __attribute__((aligned(16))) float tile[4][TS];
    __shared__ uint32_t zmask[4][TS / 32];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t C = nchunks(d);
    float* tl = tile[wv];
    const int64_t nb = (n + 63) / 64;
    for (int64_t t = (int64_t)blockIdx.x * 4 + wv; t < C * PARTS; t += (int64_t)gridDim.x * 4) {
        const int64_t c = t / PARTS;
        const uint32_t pbase = (uint32_t)((t % PARTS) * TS);
        const int64_t cbase = c * CHUNK;
        const uint32_t clen = (uint32_t)min((int64_t)CHUNK, d - cbase);
        for (int i = lane; i < TS; i += 64) tl[i] = -0.f;     // the additive identity
        constexpr int AP = RK_AP;                             // rows in flight (their gathers)
        uint32_t ro[AP];                                      // ring: part-local column (>= TS: none)
        float rv[AP];                                         //       gathered x
        // row q of the current batch: its members' columns for this lane, one gather in flight
        auto fetch = [&](const RkMeta& mt, int q, int slot) {
            const uint32_t m = __builtin_amdgcn_readlane(mt.m, q);
            // readlane returns int: widen through uint32_t (a sign-extended low word would set the high one)
            const uint64_t k = join64((uint32_t)__builtin_amdgcn_readlane(mt.khi, q), (uint32_t)__builtin_amdgcn_readlane(mt.klo, q));
            const float* rp = (const float*)join64((uint32_t)__builtin_amdgcn_readlane(mt.phi, q),
                                                   (uint32_t)__builtin_amdgcn_readlane(mt.plo, q));
            const rktree::ChunkPerm P(k, c, clen);
            uint32_t col = (uint32_t)lane < m ? P((uint32_t)lane) : NOCOL;
            if (PARTS > 1 && col - pbase >= (uint32_t)TS) col = NOCOL;   // another wave's part: no gather
            const auto rs = chunk_rsrc(rp ? rp : rows.base, cbase, d);
            ro[slot] = col - pbase;
            rv[slot] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(col * 4u), 0, 0));
        };
        auto fold = [&](int slot, float wi) {
            const uint32_t loc = ro[slot];
            if (loc < (uint32_t)TS) tl[loc] = tl[loc] + wi * (scale * rv[slot]);
        };
        RkMeta cur = rk_meta(rows, cnt, ckey, w, c, n, lane, clen), nxt;
#pragma unroll
        for (int q = 0; q < AP; ++q) fetch(cur, q, q);
        for (int64_t b = 0; b < nb; ++b) {
            const int64_t i0 = b * 64;
            nxt = rk_meta(rows, cnt, ckey, w, c, n, i0 + 64 + lane, clen);
            if (__builtin_expect(__ballot(cur.m > 64u) == 0ull, 1)) {
#pragma unroll
                for (int q = 0; q < 64; ++q) {
                    const int slot = q % AP;
                    fold(slot, __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(cur.w), q)));
                    if (q + AP < 64) fetch(cur, q + AP, slot);
                    else fetch(nxt, q + AP - 64, slot);
                }
            } else {
                // a row with more than 64 members here: the same walk with its tail folded in place
                for (int q = 0; q < 64; ++q) {
                    const int slot = q % AP;
                    const float wi = __shfl(cur.w, q, WAVE);
                    uint32_t lo = NOCOL;
                    float vv = 0.f;
#pragma unroll
                    for (int z = 0; z < AP; ++z)
                        if (z == slot) { lo = ro[z]; vv = rv[z]; }
                    if (lo < (uint32_t)TS) tl[lo] = tl[lo] + wi * (scale * vv);
                    const uint32_t m = __shfl(cur.m, q, WAVE);
                    if (m > 64u) {
                        const int64_t row = i0 + q;
                        const rktree::ChunkPerm P(ckey[row], c, clen);
                        const float* rp = rows.row(row);
                        for (uint32_t e = 64u + lane; e < m; e += 64) {
                            const uint32_t col = P(e), l2 = col - pbase;
                            if (l2 < (uint32_t)TS) tl[l2] = tl[l2] + wi * (scale * rp[cbase + col]);
                        }
                    }
                    // refill the slot (same contract as the straight-line path)
                    const RkMeta& mt = (q + AP < 64) ? cur : nxt;
                    const int qq = (q + AP) & 63;
                    const uint32_t mn = __shfl(mt.m, qq, WAVE);
                    const uint64_t kn = join64((uint32_t)__shfl(mt.khi, qq, WAVE), (uint32_t)__shfl(mt.klo, qq, WAVE));
                    const float* rpn = (const float*)join64((uint32_t)__shfl(mt.phi, qq, WAVE), (uint32_t)__shfl(mt.plo, qq, WAVE));
                    const rktree::ChunkPerm Pn(kn, c, clen);
                    const uint32_t col = (uint32_t)lane < mn ? Pn((uint32_t)lane) : NOCOL;
                    const float xv = col < clen ? rpn[cbase + col] : 0.f;
#pragma unroll
                    for (int z = 0; z < AP; ++z)
                        if (z == slot) { ro[z] = col - pbase; rv[z] = xv; }
                }
            }
            cur = nxt;
        }
        const int64_t len = min((int64_t)TS, (int64_t)clen - (int64_t)pbase);
        rk_resolve_neg_zero<TS>(tl, zmask[wv], cnt, ckey, c, n, pbase, clen, len, w, lane);
        for (int64_t i = lane; i < len; i += 64) out[cbase + pbase + i] = tl[i] / wt;
    }
}

// Single row (compressVector): out = 0, then each wave writes the members of its chunks
__global__ __launch_bounds__(256) void k_randk_scatter_dev(const float* __restrict__ x, int64_t d, const uint32_t* cnt,
                                                           const uint64_t* ckey, float scale, float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t C = nchunks(d);
    const uint64_t k = ckey[0];
    for (int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) / 64; c < C; c += (int64_t)gridDim.x * 4) {
        const int64_t cbase = c * CHUNK;
        const uint32_t clen = (uint32_t)min((int64_t)CHUNK, d - cbase);
        const rktree::ChunkPerm P(k, c, clen);
        const uint32_t m = min(cnt[c], clen);
        for (uint32_t t = (uint32_t)lane; t < m; t += 64) {
            const int64_t j = cbase + P(t);
            out[j] = scale * x[j];
        }
    }
}

// Single-row dense output (compressVector: out = zeros; out[admitted] = x, stored not added, so a
// selected -0.0 stays -0.0 like torch's out[ind] = x[ind]): after a memset, the row's list
// (entries [0, rowcnt), distinct indices) is scattered with the fold's admission rule — no per-chunk
// tile walk for one row.
__global__ __launch_bounds__(256) void k_assign_scatter(SelWs ws, float* __restrict__ out, int sharded) {
    const uint32_t T = ws.thr[0], f = ws.flags[0];
    const uint32_t mode = (f & F_EXACT) ? 2u : ((f & F_TIES) ? 1u : 0u);
    const uint32_t cut = mode == 1u ? tie_pref(ws.tiecut[0], ws.tie_hi) : 0u;
    // the list: [0, rowcnt) (one reservation counter, or rewritten by the exact path), else the
    // filter's CS_SH shards, block b taking shards b, b + gridDim.x, ...
    const bool shd = sharded && mode != 2u;
    const int64_t segcap = (ws.cap / CS_SH) & ~int64_t(3);
    for (int sh = shd ? (int)blockIdx.x : 0; sh < (shd ? CS_SH : 1); sh += shd ? (int)gridDim.x : 1) {
        const uint32_t cnt = shd ? ws.shcnt[sh * RCS] : ws.rowcnt[0];
        const int64_t o = shd ? sh * segcap : 0;
        for (uint32_t e = (shd ? 0u : blockIdx.x * 256u) + threadIdx.x; e < cnt; e += shd ? 256u : gridDim.x * 256u) {
            const uint32_t ix = ws.ent_idx[o + e];
            const float v = ws.ent_val[o + e];
            const uint32_t key = mag_key(v);
            if (mode == 2u || key > T || (key == T && tie_pref(ix, ws.tie_hi) >= cut)) out[ix] = v;
        }
    }
}

// A lone compressVector row on the fast path (its output zeroed by the filter): the exact fallback and
// the scatter in ONE launch.  A failed row (overflow / short list / ambiguous ties) is selected
// exactly by workgroup 0, which then scatters the rewritten list alone; otherwise every workgroup
// scatters its shards as k_assign_scatter does.
template <bool VEC>
__global__ __launch_bounds__(EX_NT) void k_assign_finish(RowSrc rows, int64_t d, int64_t K, SelWs ws, float* __restrict__ out) {
    __shared__ uint32_t h[HBINS];
    __shared__ uint32_t scratch[260];
    __shared__ uint32_t wsum[EX_NT / 64];
    if (ws.flags[0] & (F_OVERFLOW | F_SHORT)) {                          // uniform over the grid
        if (blockIdx.x != 0) return;
        exact_row<VEC>(rows, 1, 0, d, K, ws, h, scratch, wsum);
        __threadfence_block();
        const uint32_t cnt = ws.rowcnt[0];
        for (uint32_t e = threadIdx.x; e < cnt; e += EX_NT) out[ws.ent_idx[e]] = ws.ent_val[e];
        return;
    }
    const uint32_t T = ws.thr[0], f = ws.flags[0];
    const uint32_t cut = (f & F_TIES) ? tie_pref(ws.tiecut[0], ws.tie_hi) : 0u;
    const int64_t segcap = (ws.cap / CS_SH) & ~int64_t(3);
    for (int sh = (int)blockIdx.x; sh < CS_SH; sh += (int)gridDim.x) {
        const uint32_t cnt = ws.shcnt[sh * RCS];
        const int64_t o = sh * segcap;
        for (uint32_t e = threadIdx.x; e < cnt; e += EX_NT) {
            const uint32_t ix = ws.ent_idx[o + e];
            const float v = ws.ent_val[o + e];
            const uint32_t key = mag_key(v);
            if (key > T || (key == T && tie_pref(ix, ws.tie_hi) >= cut)) out[ix] = v;
        }
    }
}

// ------------------------------------------------------------------------------------------
// A lone compressVector row held in the chip's registers: the exact selection in ONE launch.
// The row (up to RS_U float4 a thread x 1024 threads x one workgroup per CU: 16.7 M elements on 256
// CUs, 64 MB of the chip's 128 MB of VGPRs) is read once into registers; the exact radix select
// (11/11/9-bit digits of the magnitude key, exact_row's digits) runs over it: per digit, each
// workgroup's LDS histogram is added into its group's replica (RS_NG groups: the atomics on one
// address come from G / RS_NG workgroups, not G — one global histogram's hot bins serialised 245
// deep), the workgroups arrive through a two-level counter tree, and the last to arrive sums the
// replicas, picks the digit (hist_find) and releases the others with the result in the release
// word.  After two digits the elements sharing the K-th key's 22-bit prefix (~70 on a Gaussian
// 10 M row, at most RS_CAP) are listed and ranked by the last workgroup to arrive (key, then tie
// order), which stores the kept ones; everyone else has written its dense output (x where the
// prefix is above, +0 elsewhere) and left.  Rows with more elements at that prefix take the third
// digit and a tie-rank exchange (workgroups publish their tie counts, tagged by the call's sequence
// number; one holding ties sums those before it).  No sample, no candidate lists, no fallback.
// The grid is meant to be co-resident: one 1024-thread workgroup per CU, G <= CUs, and the
// launches are serialised across the library's streams (select.hip host code).  Nothing outside
// the library is: another process's kernels, RCCL's, or a long kernel on a stream of the caller's
// can hold CUs while the grid starts.  So a wait never trusts stale data.  A wait past `spin`
// ticks of the 100 MHz clock (FLC_RS_SPIN, 0.1 s) ABORTS the call: it stores the call's sequence
// number in RS_GAVE, and every workgroup that waits (or later finds the word set) leaves without
// storing anything; a workgroup only stores output from a completed round, so every store made is
// a final value.  Every workgroup counts itself out on its group's RS_XGRP counter (after its last
// wait, before its stores; counters that run on across calls, the host passing the count before
// the launch).  The FIRST workgroup to abort instead waits for all the others to be out, then
// selects the row exactly on its own (rs_repair: three radix passes over the row in HBM and the
// dense output with the tie ranks, a few ms), rewrites the whole output, puts the control block
// back to zero and flags the row F_REPAIR.  Correct bits in every case; a clean call pays one
// non-returning counter atomic per workgroup.
// The control block is the library's own, zeroed once; a clean call leaves it clean
// (self-resetting barrier counters, replicas cleared by their merger), an aborted one is zeroed by
// its repair.
// ------------------------------------------------------------------------------------------
constexpr int RS_NT = 1024;
#ifndef FLC_RS_SPIN
#define FLC_RS_SPIN 10000000ull          // 0.1 s of the 100 MHz clock
#endif

struct RsTree {
    uint32_t* ctl;
    uint32_t grp, gsz, ngr;             // this workgroup's group, its size, groups in use
};
// The release word (64 bits at RS_GEN): generation mod 8 | a 61-bit payload, the merger's result, so
// that the waiters get it with the release itself.  A digit's payload: bin | the count above it << 11
// (24 bits: < K <= 2^24) | the bin's count << 35 (25 bits).
__device__ inline uint64_t rs_digit(uint32_t bin, uint32_t above, uint32_t last) {
    return (uint64_t)bin | ((uint64_t)above << 11) | ((uint64_t)last << 35);
}
// Self-resetting two-level barrier (no per-call clearing): a group's counter is reset by its last
// arriver, the global one by the last group's; every workgroup reads the release word BEFORE
// arriving and waits for its generation to change (the merger bumps it after every arrival, so no
// workgroup can have read the new one).  rs_arrive returns true on the last workgroup to arrive (the
// merger), whose thread 0 has acquired every other workgroup's writes.
// (gen: the release word's generation, read by thread 0 before this workgroup's flush — any time
// after the previous release — so that its load is not one more round trip here)
__device__ inline uint32_t rs_gen(const RsTree& tr) {
    return (uint32_t)__hip_atomic_load(reinterpret_cast<const uint64_t*>(tr.ctl + RS_GEN), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 7u;
}
__device__ inline bool rs_arrive(const RsTree& tr, uint32_t* flag_s, uint32_t* gen_s, uint32_t gen) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                     // this wave's atomics performed
    __syncthreads();
    if (threadIdx.x == 0) {
        *gen_s = gen;
        if (FLC_RS_FENCE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        uint32_t last = 0;
        uint32_t* gc = tr.ctl + RS_GRP + 32 * tr.grp;
#if FLC_RS_FENCE
        if (__hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == tr.gsz - 1u) {
            // the group's members' writes (released before their arrivals) ordered before this
            // workgroup's release into the global counter: acquire, then release (transitivity)
            if (FLC_RS_GACQ) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            if (__hip_atomic_fetch_add(tr.ctl + RS_GLOB, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == tr.ngr - 1u) {
                __hip_atomic_store(tr.ctl + RS_GLOB, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                last = 1;
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            }
        }
#else
        // Write-through hand-off: every member drained its atomics before its add, so when an add
        // RETURNS the members counted before it have their bytes at the coherence point, and a
        // group's last add comes before that workgroup's global add (it waits for the value).
        // The counters are never stored to: an arrival is the last of its round when it takes the
        // count to a multiple of the group size, and that workgroup takes the group size back off
        // with an add — adds commute, so whenever that add lands (before or among the next
        // round's arrivals, which start only after this round's release) the next round's
        // arrivals still return every residue mod the size once, the last one gsz - 1.
        const uint32_t o = __hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((o + 1u) % tr.gsz == 0u) {
            __hip_atomic_fetch_add(gc, 0u - tr.gsz, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t og = __hip_atomic_fetch_add(tr.ctl + RS_GLOB, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((og + 1u) % tr.ngr == 0u) {
                __hip_atomic_fetch_add(tr.ctl + RS_GLOB, 0u - tr.ngr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                last = 1;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");              // (compiler order only)
#endif
        *flag_s = last;
    }
    __syncthreads();
    return *flag_s != 0u;
}
// the merger, after its writes: the release word with its result
__device__ inline void rs_release(const RsTree& tr, const uint32_t* gen_s, uint64_t payload) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        // (the waiters read nothing but this word: its payload is the round's result)
        if (FLC_RS_FENCE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_store(reinterpret_cast<uint64_t*>(tr.ctl + RS_GEN), (uint64_t)((*gen_s + 1u) & 7u) | (payload << 3),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
// everyone else: the release word (thread 0 leaves its payload in res_s[0..1], low word first).
// false when the call is aborted — this wait passed `spin` ticks (it aborts the call; the first
// workgroup to abort, *rep_s = 1, repairs it) or another workgroup's did (RS_GAVE holds the
// call's sequence number): the caller leaves at once.
__device__ inline bool rs_wait(const RsTree& tr, const uint32_t* gen_s, uint32_t* res_s, uint32_t* ok_s,
                               uint32_t* rep_s, uint64_t spin, uint32_t seq, bool raw_bar = false) {
    if (threadIdx.x == 0) {
        const uint64_t* rw = reinterpret_cast<const uint64_t*>(tr.ctl + RS_GEN);
        uint32_t* ab = tr.ctl + RS_GAVE;
        const uint64_t t0 = (uint64_t)wall_clock64();
        uint64_t w;
        uint32_t ok = 1;
        for (uint32_t it = 0;; ++it) {
            // the abort word every FLC_RS_POLLAB-th poll (loaded beside the release word)
            w = __hip_atomic_load(rw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t a = (it % FLC_RS_POLLAB) == FLC_RS_POLLAB - 1
                                   ? __hip_atomic_load(ab, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
            if (((uint32_t)w & 7u) != *gen_s) break;
            if (a == seq) { ok = 0; break; }
            __builtin_amdgcn_s_sleep(1);
            if ((uint64_t)wall_clock64() - t0 > spin) {
                if (__hip_atomic_exchange(ab, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != seq) *rep_s = 1;
                ok = 0;
                break;
            }
        }
        if (FLC_RS_FENCE || !ok) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");      // (compiler order only)
        res_s[0] = (uint32_t)(w >> 3);
        res_s[1] = (uint32_t)(w >> 35);
        *ok_s = ok;
    }
    if (raw_bar) {                     // (the other waves' stores in flight stay in flight)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    } else {
        __syncthreads();
    }
    return *ok_s != 0u;
}

// The repair of an aborted call, by the last workgroup to leave (every other one has gone, none
// stores anything any more except final values): the control block back to zero, then the row
// selected exactly on its own — three radix passes (exact_row's 11/11/9-bit digits) over the row
// in HBM, the elements at the K-th key ranked in index order (tie rule `tie_hi`) — and the whole
// dense output written: the same function of the row as the resident selection, bit for bit.
// (32-bit indices: d * 4 < 2^31; the row state words st[0..3] = thr, krem, tiecut, flags.)
__device__ inline void rs_repair(const float* x, uint32_t d, uint32_t K, uint32_t tie_hi, uint32_t* st_thr,
                                 uint32_t* st_krem, uint32_t* st_tiecut, uint32_t* st_flags, float* out,
                                 uint32_t* ctl, uint32_t* h, uint32_t* scratch, uint32_t* wsum) {
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
    constexpr uint32_t RU4 = 4;                                        // float4 loads in flight a thread
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < (uint32_t)RS_CTL; i += RS_NT)                 // (RS_XGRP runs on: the host's xbase)
        if (i < (uint32_t)RS_XGRP || i >= (uint32_t)(RS_XGRP + 32 * RS_NG_MAX))
            __hip_atomic_store(ctl + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const auto rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), (short)0, (int)(d * 4u), 0x00020000);
    const auto ro = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, (int)(d * 4u), 0x00020000);
    const uint32_t d4 = (d + 3u) / 4u;
    uint32_t prefix = 0, krem = K, ties = 0;
    for (int p = 0; p < 3; ++p) {
        for (uint32_t i = t; i < (uint32_t)HBINS; i += RS_NT) h[i] = 0;
        __syncthreads();
        for (uint32_t f0 = t; f0 < d4; f0 += RU4 * RS_NT) {
            u4v q[RU4];
#pragma unroll
            for (uint32_t u = 0; u < RU4; ++u)                          // past the row: zeros, not counted
                q[u] = __builtin_amdgcn_raw_buffer_load_b128(rx, (f0 + u * RS_NT) * 16u, 0, 0);
#pragma unroll
            for (uint32_t u = 0; u < RU4; ++u)
#pragma unroll
                for (uint32_t e = 0; e < 4; ++e) {
                    const uint32_t k = q[u][e] & 0x7FFFFFFFu;
                    if ((f0 + u * RS_NT) * 4u + e < d && key_in_prefix(k, p, prefix)) atomicAdd(&h[key_bin(k, p)], 1u);
                }
        }
        __syncthreads();
        uint32_t bin, above;
        hist_find(h, krem, bin, above, scratch);
        prefix = (prefix << pass_bits(p)) | bin;
        krem -= above;
        if (p == 2) ties = h[bin];                                     // the row's keys == the K-th
        __syncthreads();
    }
    const uint32_t thr = prefix;
    const bool cut = ties > krem;
    const uint32_t from = tie_hi ? ties - krem : 0u, to = tie_hi ? ties : krem;
    uint32_t run = 0;                                                  // ties in index order so far
    for (uint32_t b = 0; b < d4; b += RS_NT) {
        const uint32_t f = b + t;
        const u4v q = __builtin_amdgcn_raw_buffer_load_b128(rx, f * 16u, 0, 0);
        uint32_t ne = 0;
#pragma unroll
        for (uint32_t e = 0; e < 4; ++e) ne += (f * 4u + e < d && (q[e] & 0x7FFFFFFFu) == thr) ? 1u : 0u;
        uint32_t tot;
        uint32_t r = run + ex_scan<RS_NT>(ne, wsum, tot);
        u4v o;
#pragma unroll
        for (uint32_t e = 0; e < 4; ++e) {
            const uint32_t k = q[e] & 0x7FFFFFFFu;
            const bool eq = f * 4u + e < d && k == thr;
            const bool keep = k > thr || (eq && (!cut || (r >= from && r < to)));
            r += eq ? 1u : 0u;
            o[e] = keep ? q[e] : 0u;
        }
        if (f < d4) __builtin_amdgcn_raw_buffer_store_b128(o, ro, f * 16u, 0, 0);   // (range-checked: the row end)
        run += tot;
    }
    if (t == 0) {
        *st_thr = thr;
        *st_krem = krem;
        *st_tiecut = 0;
        *st_flags = F_RESIDENT | F_REPAIR | (cut ? F_TIES : 0u);
    }
}

#ifdef FLC_RS_PRINT                       // probe builds: phase stamps of workgroup 0 (printf)
#ifndef FLC_RS_TLK
#define FLC_RS_TLK 0, 4, 1, 2, 3, 10, 12   // the 7 stamps the timeline reports (13: the merger flag)
#endif
#define RS_STAMP(i) do { if (threadIdx.x == 0) stamp[i] = (uint64_t)wall_clock64(); } while (0)
#else
#define RS_STAMP(i) do { } while (0)
#endif
template <int RU>
__global__ __launch_bounds__(RS_NT) void k_lone_resident(RowSrc rows, int64_t d, int64_t K, SelWs ws,
                                                          float* __restrict__ out, int e4, uint32_t* __restrict__ ctl,
                                                          uint32_t seq, uint64_t spin, uint32_t xbase) {
    __shared__ uint32_t h[HBINS];
    __shared__ uint32_t scratch[260];
    __shared__ uint32_t wsum[RS_NT / 64];
    __shared__ uint32_t flag_s, gen_s, ok_s, lcnt_s;
    __shared__ uint64_t lst[RS_CAP];                                     // this workgroup's listed elements
    const uint32_t G = gridDim.x, g = blockIdx.x, t = threadIdx.x;
#ifdef FLC_RS_PRINT
    uint64_t stamp[18] = {0};
    // every 16th call, workgroup 0 summarises the PREVIOUS call's per-workgroup timeline (complete:
    // that launch has ended), so that the stamps are of back-to-back calls, not of a cold launch
    if (g == 0 && t == 0 && (seq & 15u) == 0u && G <= 256u) {
        const uint64_t* pr = reinterpret_cast<const uint64_t*>(ctl + RS_PROBE);
        const int ks[7] = {FLC_RS_TLK};
        uint64_t s0 = ~0ull;
        for (uint32_t i = 0; i < G; ++i) { const uint64_t v = pr[i]; s0 = v < s0 ? v : s0; }
        uint32_t mg = 0;
        for (uint32_t i = 0; i < G; ++i) if (pr[7 * 256 + i]) mg = i;
        printf("rs_tl G=%u merger %u (x10ns from the first start): ", G, mg);
        for (int k = 0; k < 7; ++k) {
            uint64_t mn = ~0ull, mx = 0, sum = 0;
            for (uint32_t i = 0; i < G; ++i) {
                const uint64_t v = pr[k * 256 + i] - s0;
                mn = v < mn ? v : mn; mx = v > mx ? v : mx; sum += v;
            }
            printf("s%d %llu/%llu/%llu ", ks[k], mn, sum / G, mx);
        }
        printf("\n");
    }
#endif
    RS_STAMP(0);
    RsTree tr;
    tr.ctl = ctl;
    tr.grp = g % RS_NG;
    tr.ngr = min(G, (uint32_t)RS_NG);
    tr.gsz = (G - tr.grp + RS_NG - 1) / RS_NG;
    // Counted out after the workgroup's last wait and before its stores: one non-returning add to
    // its group's RS_XGRP counter (thread 0; one counter for the grid serialised ~245 atomics on one
    // address and held the kernel's end ~1 us).  The counters run over the library's launches on
    // this control block; the host passes xbase, the workgroups of its earlier launches, so the
    // repairer knows when this call's others are out (sum - xbase == G - 1) and a clean call needs
    // to know nothing.
    auto count_out = [&]() {
        // (after this lane's counter adds have landed: a repair zeroes the counters once all are out)
        if (t == 0 && !FLC_RS_FENCE) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (t == 0 && !FLC_RS_PROBE_NOCOUNT)
            __hip_atomic_fetch_add(ctl + RS_XGRP + 32 * tr.grp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    // what an aborted workgroup needs at its exit, stashed in LDS at the start: kept in registers to
    // the end, these arguments spilled SGPRs all through the dense stores (820 spill slots, not 81)
    struct RsExit {
        const float* x;
        float* out;
        uint32_t* ctl;
        uint32_t *thr, *krem, *tiecut, *flags;
        uint32_t d, K, tie_hi, seq, G, xbase;
        uint64_t spin;
    };
    __shared__ RsExit ex_s;
    __shared__ uint32_t rep_s;                                          // 1: this workgroup repairs the call
    if (t == 0) {
        rep_s = 0;
        lcnt_s = 0;
        ex_s = RsExit{rows.row_s(0), out, ctl, ws.thr, ws.krem, ws.tiecut, ws.flags, (uint32_t)d, (uint32_t)K, ws.tie_hi, seq,
                      G, xbase, spin};
    }
    const uint32_t nb = (uint32_t)(d * 4);                               // d <= RS_U * 4096 * CUs
    // the output's descriptor, rebuilt where the stores are from the LDS copy of the arguments (one
    // kept from here to the end of the kernel was spilled and shuffled around every store)
    auto out_rsrc = [&]() {
        const uint64_t op = reinterpret_cast<uint64_t>(ex_s.out);
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)op), hi = __builtin_amdgcn_readfirstlane((uint32_t)(op >> 32));
        const uint32_t nbx = __builtin_amdgcn_readfirstlane(ex_s.d * 4u);
        return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<float*>(((uint64_t)hi << 32) | lo), (short)0, (int)nbx, 0x00020000);
    };
    // float4 u of this thread: elements 4 (g e4 RS_NT + u RS_NT + t) + q, coalesced over the threads;
    // index order inside the workgroup is (u, t, q), workgroups in order (G = ceil(d / (4 e4 RS_NT))).
    // A thread's float4 u < uv lie (at least partly) inside the row; the rest are skipped.  The one
    // float4 that straddles the row end holds pad = (-d) mod 4 elements of +0 (the range-checked
    // load): padding at the END of the index order, taken out of the counts of key 0 (bin 0 while
    // the digits so far are 0; the tie count of the workgroup holding it when the K-th key is 0),
    // never stored.  (Whole padding float4 counted into bin 0 serialised ~40 K LDS atomics on one
    // address in the last workgroups: 40 us.)
    const uint32_t f0 = g * (uint32_t)e4 * RS_NT + t;                   // float4 index of u = 0
    const int64_t d4 = (d + 3) / 4;                                      // float4 touching the row
    const int uv = (int)min((int64_t)e4, max((int64_t)0, (d4 - (int64_t)f0 + RS_NT - 1) / RS_NT));
    const uint32_t pad = (uint32_t)((4 - (d & 3)) & 3);
    const uint32_t padg = (uint32_t)((d / 4) / ((int64_t)e4 * RS_NT));  // the workgroup holding it
    const uint32_t voff = f0 * 16u;
    // the speculative first digit (rows of >= 4 RS_SS elements): a fixed sample of RS_SS elements
    // (32 spread pieces of 256), the same in every workgroup, loaded BEFORE the row so that it lands
    // first (vmcnt retires in order) and its digit is picked while the row streams in
    const bool spec = FLC_RS_SPEC && d >= 4 * (int64_t)RS_SS;
    // the release word's generation for the first round, loaded before everything else (by every
    // thread, unconditionally): its wait then does not drain the row's loads (vmcnt is in order)
    // (raw: the generation is masked out where it is used, so nothing waits for this load early)
    const uint64_t gen_word = __hip_atomic_load(reinterpret_cast<const uint64_t*>(ctl + RS_GEN), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the sample's loads unconditionally (an empty descriptor when there is no speculation: zeros,
    // no memory access), so that no branch makes the compiler wait for them before the row's loads
    const int64_t spos = spec ? (int64_t)(t >> 5) * (d - 256) / 31 + (int64_t)(t & 31) * 8 : 0;
    const auto rsm = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(rows.row_s(0)), (short)0, spec ? (int)nb : 0, 0x00020000);
    const auto sa = __builtin_amdgcn_raw_buffer_load_b128(rsm, (uint32_t)(spos * 4), 0, 0);
    const auto sb = __builtin_amdgcn_raw_buffer_load_b128(rsm, (uint32_t)(spos * 4 + 16), 0, 0);
    // the workgroup's part through a descriptor of its own extent: the loads past it (u >= e4, the
    // row end) return zeros without touching memory, so all RU are issued unconditionally and the
    // compiler's in-order vmcnt count stays exact (the sample's wait does not drain the row)
    const int64_t gb = (int64_t)g * e4 * RS_NT * 4;
    const auto rxg = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(rows.row_s(0)) + gb, (short)0,
                                                       (int)(min((int64_t)e4 * RS_NT * 4, d - gb) * 4), 0x00020000);
    float4 v[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
        const auto q = __builtin_amdgcn_raw_buffer_load_b128(rxg, t * 16u, u * RS_NT * 16, FLC_LOADPOL);
        v[u] = make_float4(__uint_as_float(q[0]), __uint_as_float(q[1]), __uint_as_float(q[2]), __uint_as_float(q[3]));
    }
#ifdef FLC_RS_PRINT
    if (t < 64) {                                                        // (probe: when wave 0's row has landed)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        RS_STAMP(4);
    }
#endif
#if defined(FLC_RS_EXIT) && FLC_RS_EXIT == 3                             // (cost probe: the loads, then the row stored)
    {
        typedef unsigned int u4v __attribute__((ext_vector_type(4)));
        const uint64_t op = reinterpret_cast<uint64_t>(out);
        const auto rq = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<float*>(op), (short)0, (int)nb, 0x00020000);
#pragma unroll
        for (int u = 0; u < RU; ++u)
            if (u < uv) {
                const u4v ov = {__float_as_uint(v[u].x), __float_as_uint(v[u].y), __float_as_uint(v[u].z), __float_as_uint(v[u].w)};
                __builtin_amdgcn_raw_buffer_store_b128(ov, rq, voff, u * RS_NT * 16, FLC_RS_STPOL);
            }
        return;
    }
#endif
#if defined(FLC_RS_EXIT) && FLC_RS_EXIT == 1                             // (cost probe: the loads only)
    {
        uint32_t a = 0;
#pragma unroll
        for (int u = 0; u < RU; ++u) a |= __float_as_uint(v[u].x);
        if (a == 0x7FFFFFFFu) out[0] = 1.f;
        return;
    }
#endif
    uint32_t prefix = 0, krem = (uint32_t)K, last = 0, bar = 0;
    bool cand = false;
    uint32_t bs = 0;
    int p0 = 0;
    // bit u: float4 u holds an element whose first digit is in the speculative window (bs +- 1);
    // the others were stored before the round's release when the guess hits (FLC_RS_SPECST)
    uint32_t winm = 0;
    bool sst = false;                                                    // (uniform) those stores made and final
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
    if (spec) {
        __shared__ uint32_t h1[3 * HBINS];
        // the sample's first-digit histogram in RS_SR replicas, lane l adding to replica l mod
        // RS_SR (a padded stride: other banks) — the exponents crowd a Gaussian row's keys into a
        // few bins; but the conflicts are not on the path (8 replicas: 0.35 us slower a call)
        __shared__ uint32_t hs[RS_SR * (HBINS + 1)];
        const uint32_t gen = (uint32_t)gen_word & 7u;
        // (LDS-only barriers up to the row's histogram: the sample's digit is picked while the
        // row's loads are still in flight — a __syncthreads waits for them, ~7 us)
        for (int i = t; i < RS_SR * (HBINS + 1); i += RS_NT) hs[i] = 0;
        for (int i = t; i < 3 * HBINS; i += RS_NT) h1[i] = 0;
        lds_bar();
        {
            uint32_t* hr = hs + (t % RS_SR) * (HBINS + 1);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                atomicAdd(&hr[(sa[q] & 0x7FFFFFFFu) >> 20], 1u);
                atomicAdd(&hr[(sb[q] & 0x7FFFFFFFu) >> 20], 1u);
            }
        }
        lds_bar();
        for (int i = t; i < HBINS; i += RS_NT) {
            uint32_t c = 0;
#pragma unroll
            for (int r = 0; r < RS_SR; ++r) c += hs[r * (HBINS + 1) + i];
            h[i] = c;
        }
        lds_bar();
        RS_STAMP(5);
#if defined(FLC_RS_EXIT) && FLC_RS_EXIT == 2                             // (cost probe: loads + the sample's digit)
        if (h[t] == 0x7FFFFFFFu) out[0] = 1.f;
        return;
#endif
        uint32_t ab;
        const uint32_t rs = (uint32_t)min((int64_t)RS_SS, max((int64_t)1, (K * RS_SS + d / 2) / d));
        hist_find<true>(h, rs, bs, ab, scratch);                         // the sample's digit (uniform)
        lds_bar();
        RS_STAMP(6);
        // the second digit's histograms for the first digits bs - 1 .. bs + 1, and the count of keys
        // whose first digit is above them: with the K-th key's first digit among the three, that is
        // all the merger needs for both digits (the contended first-digit histogram — the exponents
        // crowd into few bins — is not built at all unless the guess misses)
        uint32_t km = 0x7FFFFFFFu;
        asm volatile("" : "+s"(km));
        // (per element: the key, its offset from the window's low end, one compare into the
        // histogram's exec mask, one into a ballot counted by the scalar unit — every VALU op a
        // row element costs is ~0.25 us of a launch with one 16-wave workgroup per CU)
        const uint32_t wlo = (bs - 1u) << 20, whi = (bs + 2u) << 20;   // the window: first digits bs-1 .. bs+1
        uint32_t abv = 0;                                                // keys above the window (wave total)
#pragma unroll
        for (int u = 0; u < RU; ++u) {
            if (u < uv) {
                const float e[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t k = __float_as_uint(e[q]) & km;
                    const uint32_t dd = k - wlo;                         // window bin = dd >> 9 (3 x 2048)
                    abv += (uint32_t)__popcll(__ballot(k >= whi));
                    if (dd < (3u << 20)) {
                        atomicAdd(&h1[dd >> 9], 1u);
                        winm |= 1u << u;
                    }
                }
            }
        }
        RS_STAMP(7);
        if (t == 0) scratch[0] = 0;
        __syncthreads();
        if ((t & 63) == 0 && abv) atomicAdd(&scratch[0], abv);
        __syncthreads();
        RS_STAMP(1);
#if defined(FLC_RS_EXIT) && FLC_RS_EXIT == 4                             // (cost probe: + the window histograms)
        if (scratch[0] == 0x7FFFFFFFu) out[0] = 1.f;
        return;
#endif
        // the float4 with no element in the window: final if the guess hits (first digit above the
        // window: kept, below: +0), stored while the round runs; a miss rewrites every float4 later
        auto spec_store = [&]() {
            if (!FLC_RS_SPECST) return;
            const auto ro = out_rsrc();
            // (opaque copies: the 16 per-float4 lane masks the compiler would otherwise compute
            // once and keep for the later store loops spilled SGPRs through the whole kernel)
            int uvx = uv;
            uint32_t wmx = winm;
            asm volatile("" : "+v"(uvx), "+v"(wmx));
#pragma unroll
            for (int u = 0; u < RU; ++u) {
                if (u < uvx && !((wmx >> u) & 1u)) {
                    const float e[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
                    uint32_t o[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) o[q] = (mag_key(e[q]) >> 20) > bs + 1u ? __float_as_uint(e[q]) : 0u;
                    const u4v ov = {o[0], o[1], o[2], o[3]};
                    // (the float4's offset in the VGPR operand: 16 scalar offsets kept live here
                    // spilled SGPRs through the whole kernel)
                    __builtin_amdgcn_raw_buffer_store_b128(ov, ro, voff + (uint32_t)(u * RS_NT * 16), 0, FLC_RS_STPOL);
                }
            }
        };
        uint32_t* gs = ctl + RS_HSPEC + tr.grp * 3 * HBINS;
        for (int i = t; i < 3 * HBINS; i += RS_NT)
            if (h1[i]) __hip_atomic_fetch_add(gs + i, h1[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t == 0 && scratch[0]) __hip_atomic_fetch_add(ctl + RS_ABV + 32 * tr.grp, scratch[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ++bar;
        // (the speculative stores: by the waves 1.. of the workgroups that wait, while they wait —
        // wave 0 polls, and a poll would queue behind stores of its own, so it stores all its
        // float4 at the end; the merger's after its release, its loads not queued behind them)
        if (FLC_RS_SPECST && t < 64) winm = 0xFFFFu;
        const bool mg_ = rs_arrive(tr, &flag_s, &gen_s, gen);
#if defined(FLC_RS_EXIT) && FLC_RS_EXIT == 5                             // (cost probe: + the flush and the arrival)
        return;
#endif
        if (mg_) {
            // the merger: the three second-digit histograms summed (all loads in flight at once) with
            // their totals; the first digit is the one of the three where the count from the top
            // reaches K (else the guess missed: the rounds start from the first digit), the second
            // from its histogram — both digits in ONE round
            RS_STAMP(2);
#ifdef FLC_RS_PRINT
            stamp[13] = 1;
#endif
            // every replica word loaded at once (RS_NG x 3 x HBINS / RS_NT a thread, one round trip),
            // then added into h1 (its own counts first cleared) by LDS atomics
            uint32_t* s0 = ctl + RS_HSPEC;
            constexpr int ML = RS_NG * 3 * HBINS / RS_NT;
            uint32_t mv[ML];
#pragma unroll
            for (int j = 0; j < ML; ++j) mv[j] = __hip_atomic_load(s0 + t + j * RS_NT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t ar = t < RS_NG ? __hip_atomic_load(ctl + RS_ABV + 32 * t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
            for (int i = t; i < 3 * HBINS; i += RS_NT) h1[i] = 0;
            __syncthreads();
#pragma unroll
            for (int j = 0; j < ML; ++j) {
                const int i = (t + j * RS_NT) % (3 * HBINS);
                if (mv[j]) atomicAdd(&h1[i], mv[j]);
            }
            if (t < 64) {
                const uint32_t a4 = wave_sum(ar);
                if (t == 0) scratch[259] = a4;
            }
            __syncthreads();
            if (t < 2) {                                                 // the padding: first digit 0, second 0
                if (bs + (uint32_t)t == 1u) h1[t * HBINS] -= pad;
            }
            __syncthreads();
            const uint32_t A = scratch[259];
            // the three windows in index order w 0, 1, 2 are first digits bs - 1, bs, bs + 1: from the
            // top, h1's 3 x 2048 bins descend through both digits at once — one search finds both
            uint32_t bb = 0, ab = 0;
            bool found = false;
            if (A < (uint32_t)K) hist_find_n<3 * HBINS>(h1, (uint32_t)K - A, bb, ab, found, scratch);   // (uniform)
            uint64_t pl = 0;                                             // miss: start from the first digit
            if (found) {
                const uint32_t w0 = bb / HBINS, b1 = bb % HBINS, b0 = bs - 1u + w0;
                // hit | 22-bit prefix << 1 | krem << 23 | the prefix's count (saturated) << 47
                pl = 1ull | ((uint64_t)((b0 << 11) | b1) << 1) | ((uint64_t)((uint32_t)K - A - ab) << 23) |
                     ((uint64_t)min(h1[bb], 16383u) << 47);
            }
            rs_release(tr, &gen_s, pl);
            if (t == 0) { scratch[0] = (uint32_t)pl; scratch[1] = (uint32_t)(pl >> 32); }
            RS_STAMP(3);
            spec_store();
            if (t < RS_NG) __hip_atomic_store(ctl + RS_ABV + 32 * t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (int i = t; i < 3 * RS_NG * HBINS; i += RS_NT)           // clean for the next call
                __hip_atomic_store(s0 + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            RS_STAMP(2);
            spec_store();
            if (!rs_wait(tr, &gen_s, scratch, &ok_s, &rep_s, spin, seq, true)) goto leave;
        }
        // (raw barriers: a __syncthreads here would drain the speculative stores first)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        const uint64_t pl = ((uint64_t)scratch[1] << 32) | scratch[0];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (pl & 1u) {
            prefix = (uint32_t)(pl >> 1) & 0x3FFFFFu;
            krem = (uint32_t)(pl >> 23) & 0xFFFFFFu;
            last = (uint32_t)(pl >> 47);
            p0 = 2;
            cand = last <= (uint32_t)RS_CAP;
            sst = FLC_RS_SPECST;
        }
#if defined(FLC_RS_EXIT) && FLC_RS_EXIT == 6                             // (cost probe: + the merger and the release)
        return;
#endif                                                                // (else p0 = 0: the full rounds)
        RS_STAMP(3);
    }
    for (int p = p0; p < 3 && !cand; ++p) {
        const uint32_t gen = (p == 0 && !spec) ? ((uint32_t)gen_word & 7u) : (t == 0 ? rs_gen(tr) : 0u);
        for (int i = t; i < HBINS; i += RS_NT) h[i] = 0;
        __syncthreads();
        // an opaque copy of the key mask per pass: keeps the compiler from hoisting the 4 RU keys out
        // of the pass loop into as many more VGPRs (spills at 128)
        uint32_t km = 0x7FFFFFFFu;
        asm volatile("" : "+s"(km));
#pragma unroll
        for (int u = 0; u < RU; ++u) {
            if (u < uv) {
                const float e[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t k = __float_as_uint(e[q]) & km;
                    if (key_in_prefix(k, p, prefix)) atomicAdd(&h[key_bin(k, p)], 1u);
                }
            }
        }
        __syncthreads();
        RS_STAMP(1 + 3 * p);
        uint32_t* gh = ctl + RS_HREP + (p * RS_NG + tr.grp) * HBINS;
        for (int i = t; i < HBINS; i += RS_NT)
            if (h[i]) __hip_atomic_fetch_add(gh + i, h[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ++bar;
        if (rs_arrive(tr, &flag_s, &gen_s, gen)) {
            // the merger: the replicas summed, the digit picked, the result released with the
            // generation; the replicas cleared for the next call after that (off the critical path)
            RS_STAMP(2 + 3 * p);
            uint32_t* r0 = ctl + RS_HREP + p * RS_NG * HBINS;
            for (int i = t; i < HBINS; i += RS_NT) {
                uint32_t c = 0;
#pragma unroll
                for (int r = 0; r < RS_NG; ++r) c += __hip_atomic_load(r0 + r * HBINS + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                h[i] = (i == 0 && prefix == 0u) ? c - pad : c;
            }
            __syncthreads();
            uint32_t bin, above;
            hist_find(h, krem, bin, above, scratch);
            const uint64_t pl = rs_digit(bin, above, h[bin]);
            rs_release(tr, &gen_s, pl);
            if (t == 0) { scratch[0] = (uint32_t)pl; scratch[1] = (uint32_t)(pl >> 32); }
            for (int i = t; i < HBINS; i += RS_NT)
#pragma unroll
                for (int r = 0; r < RS_NG; ++r) __hip_atomic_store(r0 + r * HBINS + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            RS_STAMP(2 + 3 * p);
            if (!rs_wait(tr, &gen_s, scratch, &ok_s, &rep_s, spin, seq)) goto leave;
        }
        __syncthreads();
        const uint64_t pl = ((uint64_t)scratch[1] << 32) | scratch[0];
        const uint32_t bin = (uint32_t)pl & 0x7FFu, above = (uint32_t)(pl >> 11) & 0xFFFFFFu;
        last = (uint32_t)(pl >> 35);
        prefix = (prefix << pass_bits(p)) | bin;
        krem -= above;
        __syncthreads();
        RS_STAMP(3 + 3 * p);
        if (p == 1 && last <= (uint32_t)RS_CAP) { cand = true; break; }  // (uniform) the candidate finish
    }
    if (cand) {
        // Candidate finish (after two digits, the K-th key's 22-bit prefix P holding <= RS_CAP
        // elements): keys above P are kept, below dropped, and the elements AT P — the K-th and its
        // equals — are stored as +0 now and listed (value bits, index); the last workgroup to arrive
        // ranks the list by (key desc, tie order), stores the krem first and writes the row state.
        // The third digit's round and the tie counts' exchange are not needed; nobody waits for the
        // ranking.  (The padding of the straddling float4 is never listed.)
        const uint32_t P = prefix;
        const uint32_t plo = P << 9;                                     // keys at P: [plo, plo + 512)
        // the listed elements into this workgroup's LDS list at positions from an LDS counter
        // (~70 in a 10 M row: the rare atomics cost less than a counting pass and a scan over
        // every element), then wave 0 hands them over: the first RS_CS into this workgroup's own
        // slots (no shared counter on the path: 245 returning adds on one word serialised ~3 us),
        // any beyond them into the shared list at a reserved offset, the count into its count word
#pragma unroll
        for (int u = 0; u < RU; ++u) {
            if (u < uv) {
                const float e[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (mag_key(e[q]) - plo < 512u) {
                        const uint32_t j = (f0 + u * RS_NT) * 4u + (uint32_t)q;
                        if ((int64_t)j < d) {                            // (not the straddling float4's padding)
                            const uint32_t pp = atomicAdd(&lcnt_s, 1u);
                            if (pp < (uint32_t)RS_CAP) lst[pp] = ((uint64_t)__float_as_uint(e[q]) << 32) | j;
                        }
                    }
                }
            }
        }
        lds_bar();
        const uint32_t ctot = lcnt_s;                                    // (uniform)
        RS_STAMP(9);
        if (FLC_RS_DONE && t < 64 && ctot) {
            // (the workgroups without candidates — nearly all — store nothing here)
            uint64_t* cl = reinterpret_cast<uint64_t*>(ctl + RS_CLIST);
            uint32_t ob = 0;
            if (t == 0) ob = __hip_atomic_fetch_add(ctl + RS_CCNT, ctot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t obase = __shfl(ob, 0, 64);
            const uint32_t nl = min(ctot, (uint32_t)RS_CAP);
            for (uint32_t i = t; i < nl; i += 64)
                if (obase + i < (uint32_t)RS_CAP) __hip_atomic_store(cl + obase + i, lst[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (t == 0) __hip_atomic_fetch_add(ctl + RS_CDONE, ctot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (!FLC_RS_DONE && t < 64) {
            uint64_t* cl = reinterpret_cast<uint64_t*>(ctl + RS_CLIST);
            uint64_t* cr = reinterpret_cast<uint64_t*>(ctl + RS_CREG) + (size_t)g * RS_CS;
            uint32_t ob = 0;
            if (ctot > (uint32_t)RS_CS && t == 0)
                ob = __hip_atomic_fetch_add(ctl + RS_CCNT, ctot - (uint32_t)RS_CS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t obase = __shfl(ob, 0, 64);
            const uint32_t nl = min(ctot, (uint32_t)RS_CAP);
            for (uint32_t i = t; i < nl; i += 64) {
                const uint64_t en = lst[i];
                if (i < (uint32_t)RS_CS) __hip_atomic_store(cr + i, en, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else if (obase + i - RS_CS < (uint32_t)RS_CAP)
                    __hip_atomic_store(cl + obase + i - RS_CS, en, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (t == 0) __hip_atomic_store(ctl + RS_CNUM + g, ctot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        // the dense output without the listed positions (the ranking workgroup writes those); with
        // the speculative stores made, only the float4 holding a window element are left
        auto dense = [&]() {
            const auto ro = out_rsrc();
            int uvx = uv;
            uint32_t wmx = sst ? winm : 0xFFFFu;
            asm volatile("" : "+v"(uvx), "+v"(wmx));
#pragma unroll
            for (int u = 0; u < RU; ++u) {
                if (u < uvx && ((wmx >> u) & 1u)) {
                    const float e[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
                    uint32_t o[4];
                    bool at[4], any = false;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const uint32_t k = mag_key(e[q]);
                        o[q] = k >= plo + 512u ? __float_as_uint(e[q]) : 0u;
                        at[q] = k - plo < 512u;
                        any |= at[q];
                    }
                    if (!any) {
                        const u4v ov = {o[0], o[1], o[2], o[3]};
                        __builtin_amdgcn_raw_buffer_store_b128(ov, ro, voff, u * RS_NT * 16, FLC_RS_STPOL);
                    } else {
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            if (!at[q]) __builtin_amdgcn_raw_buffer_store_b32(o[q], ro, voff + 4u * q, u * RS_NT * 16, FLC_RS_STPOL);
                    }
                }
            }
        };
        RS_STAMP(10);
        // the hand-over drained (wave 0), then the workgroup counts out (its last hand-off) and
        // every wave stores its dense output — except the ranking workgroup (the last one: its
        // slice of the row is the shortest), which stores its dense output, waits until the
        // others are out, then ranks the list
        if (g != G - 1u) {
            count_out();
            lds_bar();                                                   // (nothing stored before the count-out)
#if defined(FLC_RS_EXIT) && FLC_RS_EXIT == 7                             // (cost probe: all but the others' dense stores)
            return;
#endif
            dense();
        } else {
            if (!FLC_RS_RANKFIRST) dense();
            // (everything below from the LDS copy of the arguments: kept in registers across the
            // dense stores they spill SGPRs all through them)
            const RsExit ex = ex_s;
            if (t == 0) {
                const uint64_t t0 = (uint64_t)wall_clock64();
                uint32_t okw = 1;
                for (;;) {
                    if (FLC_RS_DONE) {
                        // (every candidate delivered; more than `last` would be a list that does
                        // not add up: the check below aborts it)
                        if (__hip_atomic_load(ex.ctl + RS_CDONE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= last) break;
                    } else {
                        uint32_t out_n = 0;
#pragma unroll
                        for (int r = 0; r < RS_NG; ++r)
                            out_n += __hip_atomic_load(ex.ctl + RS_XGRP + 32 * r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (out_n - ex.xbase >= ex.G - 1u) break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    if ((uint64_t)wall_clock64() - t0 > ex.spin) {                 // (never seen: all ran the round)
                        if (__hip_atomic_exchange(ex.ctl + RS_GAVE, ex.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ex.seq) rep_s = 1;
                        okw = 0;
                        break;
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");          // (compiler order only)
                ok_s = okw;
            }
            __syncthreads();
            if (!ok_s) goto leave;
            // the list: every workgroup's count and slots (one thread each, all loads at once; slots
            // beyond a count are stale and unused), then the shared list's overflow entries — m
            // entries in all, every element at P (checked: a list that does not add up aborts the
            // call and the repair selects the row), ranked by (key desc, tie order)
            __shared__ uint64_t comp[RS_CAP];
            __shared__ uint64_t ent[RS_CAP];
            __shared__ uint64_t kth_s;
            uint32_t m, ns, ovn, mm;
            bool ok;
            if (FLC_RS_DONE) {
                // the shared list holds exactly the `last` candidates (delivered count and reserved
                // count agree), read in one pass
                if (t == 0) {
                    scratch[4] = __hip_atomic_load(ex.ctl + RS_CCNT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    scratch[5] = __hip_atomic_load(ex.ctl + RS_CDONE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                __syncthreads();
                m = scratch[4];
                ok = m == last && scratch[5] == last && m >= krem && krem >= 1u && m <= (uint32_t)RS_CAP;
                mm = ok ? m : 0u;
                for (uint32_t i = t; i < mm; i += RS_NT)
                    ent[i] = __hip_atomic_load(reinterpret_cast<const uint64_t*>(ex.ctl + RS_CLIST) + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ovn = 1u;                                                // (the reserved count to reset below)
            } else {
            uint32_t c = 0;
            uint64_t sl[RS_CS];
            if (t < ex.G) {
                c = __hip_atomic_load(ex.ctl + RS_CNUM + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint64_t* ct = reinterpret_cast<const uint64_t*>(ex.ctl + RS_CREG) + (size_t)t * RS_CS;
#pragma unroll
                for (int k = 0; k < RS_CS; ++k) sl[k] = __hip_atomic_load(ct + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            const uint32_t ov = t == 0 ? __hip_atomic_load(ex.ctl + RS_CCNT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
            if (t == 0) scratch[4] = ov;
            const uint32_t cs = min(c, (uint32_t)RS_CS);
            (void)ex_scan<RS_NT>(c, wsum, m);                            // (also the barrier before scratch[4])
            const uint32_t sp = ex_scan<RS_NT>(cs, wsum, ns);
            ovn = scratch[4];
            ok = m == last && ovn == m - ns && m >= krem && krem >= 1u && m <= (uint32_t)RS_CAP;
            mm = ok ? m : 0u;
            if (ok) {
#pragma unroll
                for (int k = 0; k < RS_CS; ++k)
                    if ((uint32_t)k < cs) ent[sp + k] = sl[k];
                for (uint32_t i = t; i < ovn; i += RS_NT) ent[ns + i] = __hip_atomic_load(reinterpret_cast<const uint64_t*>(ex.ctl + RS_CLIST) + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            }
            if (t == 0) { scratch[2] = 0; scratch[3] = 0; kth_s = ~0ull; }
            __syncthreads();
            for (uint32_t i = t; i < mm; i += RS_NT) {
                const uint64_t en = ent[i];
                comp[i] = ((uint64_t)((uint32_t)(en >> 32) & 0x7FFFFFFFu) << 32) | tie_pref((uint32_t)en, ex.tie_hi);
            }
            __syncthreads();
            for (uint32_t i = t; i < mm; i += RS_NT) {
                const uint64_t me = comp[i];
                uint32_t rank = 0;
                for (uint32_t jj = 0; jj < mm; ++jj) rank += comp[jj] > me ? 1u : 0u;
                if (rank == krem - 1u) kth_s = me;                       // entries are distinct
            }
            __syncthreads();
            const uint64_t kc = kth_s;
            const uint32_t kth = (uint32_t)(kc >> 32);
            for (uint32_t i = t; i < mm; i += RS_NT) {
                const uint64_t me = comp[i];
                const uint64_t en = ent[i];
                ex.out[(uint32_t)en] = me >= kc ? __uint_as_float((uint32_t)(en >> 32)) : 0.f;
                const uint32_t key = (uint32_t)(me >> 32);
                if (key > kth) atomicAdd(&scratch[2], 1u);
                else if (key == kth) atomicAdd(&scratch[3], 1u);
            }
            __syncthreads();
            if (t == 0) {
                if (ovn) __hip_atomic_store(ex.ctl + RS_CCNT, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // clean for the next call
                if (FLC_RS_DONE) __hip_atomic_store(ex.ctl + RS_CDONE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t gt = scratch[2], eq = scratch[3];
                *ex.thr = kth;
                *ex.krem = krem - gt;
                *ex.tiecut = tie_pref((uint32_t)kc, ex.tie_hi);
                *ex.flags = F_RESIDENT | (gt + eq > krem ? F_TIES : 0u);
                if (!ok && __hip_atomic_exchange(ex.ctl + RS_GAVE, ex.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ex.seq)
                    rep_s = 1;
            }
            if (!ok) goto leave;                                         // (uniform) aborted: repaired
            if (t == 0) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_fetch_add(ex.ctl + RS_XGRP + 32 * (blockIdx.x % RS_NG), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (FLC_RS_RANKFIRST) dense();
        }
        RS_STAMP(11);
    } else {
    // thr = the K-th key; krem of the `last` elements equal to it are kept
    const uint32_t thr = prefix;
    const bool tie_cut = last > krem;                                    // uniform over the grid
    uint64_t tmask = 0;                                                  // kept ties: bit 4 u + q
    if (tie_cut) {
        // this workgroup's ties (its padding, at its end, is not one), published as (call seq << 32 |
        // count); a workgroup holding ties sums the counts of the workgroups before it (waiting for
        // each to be published: all publish right after the last digit, so no barrier round) and
        // ranks its own in (u, t, q) order; the others have nothing to rank
        uint32_t c = 0;
#pragma unroll
        for (int u = 0; u < RU; ++u) {
            if (u < uv) {
                const float e[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                for (int q = 0; q < 4; ++q) c += mag_key(e[q]) == thr ? 1u : 0u;
            }
        }
        uint32_t tot;
        (void)ex_scan<RS_NT>(c, wsum, tot);
        if (thr == 0u && g == padg) tot -= pad;
        uint64_t* tc = reinterpret_cast<uint64_t*>(ctl + RS_TCNT);
        if (t == 0) __hip_atomic_store(tc + g, ((uint64_t)seq << 32) | tot, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        if (tot == 0u) goto store;                                       // (uniform) no tie here
        uint32_t part = 0, run = 0;
        int bail = 0;
        const uint64_t t0 = (uint64_t)wall_clock64();
        for (uint32_t i = t; i < g && !bail; i += RS_NT) {
            uint64_t w;
            for (;;) {
                w = __hip_atomic_load(tc + i, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t a = __hip_atomic_load(ctl + RS_GAVE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((uint32_t)(w >> 32) == seq) break;
                if (a == seq) { bail = 1; break; }                       // aborted elsewhere
                __builtin_amdgcn_s_sleep(1);
                if ((uint64_t)wall_clock64() - t0 > spin) {             // a workgroup before is not running
                    if (__hip_atomic_exchange(ctl + RS_GAVE, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != seq)
                        rep_s = 1;                                       // (one thread of the grid)
                    bail = 1;
                    break;
                }
            }
            part += (uint32_t)w;
        }
        if (__syncthreads_or(bail)) goto leave;                          // (uniform) the call is aborted
        (void)ex_scan<RS_NT>(part, wsum, run);                           // ties in the workgroups before
        const uint32_t tie_from = ws.tie_hi ? last - krem : 0u, tie_to = ws.tie_hi ? last : krem;
#pragma unroll
        for (int u = 0; u < RU; ++u) {
            if (u < e4) {                                                // (uniform: ex_scan inside)
                const float e[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
                uint32_t ce = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) ce += (u < uv && mag_key(e[q]) == thr) ? 1u : 0u;
                uint32_t tu;
                uint32_t r = run + ex_scan<RS_NT>(ce, wsum, tu);
                run += tu;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (u < uv && mag_key(e[q]) == thr) {
                        if (r >= tie_from && r < tie_to) tmask |= 1ull << (4 * u + q);
                        ++r;
                    }
            }
        }
    }
store:
    RS_STAMP(10);
    // every wait of this workgroup is behind it: the row state (workgroup 0: released before it is
    // counted out, so that a repair's later state is the one that stays), counted out, then the
    // stores (final values)
    if (g == 0 && t == 0) {
#if FLC_RS_FENCE
        ws.thr[0] = thr;
        ws.krem[0] = krem;
        ws.tiecut[0] = 0;
        ws.flags[0] = F_RESIDENT | (tie_cut ? F_TIES : 0u);
        if (FLC_RS_G0REL) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
#else
        // written through (agent-scope stores) and drained before the count-out, so that a
        // repair's later row state is the one that stays
        __hip_atomic_store(ws.thr, thr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ws.krem, krem, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ws.tiecut, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ws.flags, F_RESIDENT | (tie_cut ? F_TIES : 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    }
    count_out();
    // the dense output from the registers: x where kept, +0 elsewhere (range-checked: no padding);
    // with the speculative stores made, only the float4 holding a window element
    const auto ro = out_rsrc();
    int uvx = uv;
    uint32_t wmx = sst ? winm : 0xFFFFu;
    asm volatile("" : "+v"(uvx), "+v"(wmx));
#pragma unroll
    for (int u = 0; u < RU; ++u) {
        if (u < uvx && ((wmx >> u) & 1u)) {
            const float e[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
            uint32_t o[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t k = mag_key(e[q]);
                const bool keep = k > thr || (k == thr && (!tie_cut || ((tmask >> (4 * u + q)) & 1ull)));
                o[q] = keep ? __float_as_uint(e[q]) : 0u;
            }
            const u4v ov = {o[0], o[1], o[2], o[3]};
            __builtin_amdgcn_raw_buffer_store_b128(ov, ro, voff, u * RS_NT * 16, FLC_RS_STPOL);
        }
    }
    RS_STAMP(11);
    (void)bar;
    }
    goto done;
leave:
    // An aborted workgroup (it left from a wait, or the ranking found the list inconsistent): its
    // control-block writes completed (release), then counted out — except the repairer (the first
    // to abort), which waits for every other workgroup of the call to be out, selects the row on
    // its own, rewrites the output and the row state, zeroes the control block, then counts out.
    if (t == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    }
    if (!rep_s) count_out();
    __syncthreads();
    if (rep_s) {
        const RsExit ex = ex_s;
        if (t == 0) {
            // (bounded: every other workgroup leaves within its own waits' limit once it runs; a
            // grid that cannot drain at all after 64 of them is repaired anyway — its stragglers
            // never store anything but final values)
            const uint64_t t0 = (uint64_t)wall_clock64();
            for (;;) {
                uint32_t out_n = 0;
                for (int r = 0; r < RS_NG; ++r)
                    out_n += __hip_atomic_load(ex.ctl + RS_XGRP + 32 * r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (out_n - ex.xbase >= ex.G - 1u || (uint64_t)wall_clock64() - t0 >= 64 * ex.spin) break;
                __builtin_amdgcn_s_sleep(8);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        __syncthreads();
        rs_repair(ex.x, ex.d, ex.K, ex.tie_hi, ex.thr, ex.krem, ex.tiecut, ex.flags, ex.out, ex.ctl, h, scratch, wsum);
        __syncthreads();
        if (t == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        count_out();
    }
done:;
#ifdef FLC_RS_PRINT
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    RS_STAMP(12);
    if (t == 0 && G <= 256u) {
        uint64_t* pr = reinterpret_cast<uint64_t*>(ex_s.ctl + RS_PROBE);
        const int ks[8] = {FLC_RS_TLK, 13};
        for (int k = 0; k < 8; ++k) __hip_atomic_store(pr + k * 256 + g, stamp[ks[k]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#endif
}

// ------------------------------------------------------------------------------------------
// Host orchestration
// ------------------------------------------------------------------------------------------
static int64_t host_chunks(int64_t d) { return (d + CHUNK - 1) / CHUNK; }

int64_t sel_capacity(int codec, int64_t d, int64_t K) {
    if (codec == FLC_RANDK) return std::max<int64_t>(K, 1);
    // candidates of the fast path (~K (1 + 4/sqrt(ks))) with margin; the exact path needs K + CHUNK
    int64_t cap = 2 * K + 2 * CHUNK;
    cap = std::min<int64_t>(std::max<int64_t>(cap, 1), std::max<int64_t>(d, 1));
    return (cap + 3) & ~int64_t(3);        // rows of the candidate lists start 16 B aligned
}

static SelWs carve_sel(void* base, int codec, int64_t n, int64_t d, int64_t K, size_t* bytes) {
    Carver cv(base);
    const int64_t C = std::max<int64_t>(host_chunks(d), 1), nn = std::max<int64_t>(n, 1);
    SelWs s;
    s.tie_hi = 0;
    s.cap = sel_capacity(codec, d, K);
    s.tab = cv.take<uint2>((size_t)C * nn);
    s.ent_idx = cv.take<uint32_t>((size_t)nn * s.cap);
    s.ent_val = cv.take<float>((size_t)nn * s.cap);
    s.rowcnt = cv.take<uint32_t>((size_t)nn * RCS);
    s.flags = cv.take<uint32_t>(nn);
    s.thr = cv.take<uint32_t>(nn);
    s.prefix = cv.take<uint32_t>(nn);
    s.krem = cv.take<uint32_t>(nn);
    s.worklist = cv.take<uint32_t>(nn);
    s.nwork = cv.take<uint32_t>(4);
    s.zm = cv.take<uint32_t>((size_t)C * (CHUNK / 32));
    s.part = codec == FLC_TOPK ? cv.take<float>((size_t)C * CHUNK) : nullptr;
    if (codec == FLC_TOPK) {
        s.tieprefix = cv.take<uint32_t>((size_t)C * nn);
        s.tiecut = cv.take<uint32_t>(nn);
        s.hist = cv.take<uint32_t>((size_t)nn * HBINS);
        s.cursor = nullptr;
        s.cstate = cv.take<uint32_t>((size_t)nn * CS_ST);
        s.clist = cv.take<uint64_t>((size_t)std::min<int64_t>(nn, CS_FEW) * CS_LCAP);
        s.carrive = cv.take<uint32_t>((size_t)nn * RCS);
        s.shcnt = cv.take<uint32_t>((size_t)std::min<int64_t>(nn, CS_FEW) * CS_SH * RCS);
    } else {
        s.tieprefix = nullptr;
        s.tiecut = nullptr;
        s.hist = nullptr;
        s.cursor = cv.take<uint32_t>((size_t)std::max<int64_t>(C, RK_SB) * nn);   // RandK: [N][RK_SB] segment offsets
        s.cstate = nullptr;
        s.clist = nullptr;
        s.carrive = nullptr;
        s.shcnt = nullptr;
    }
    if (bytes) *bytes = cv.bytes();
    return s;
}

size_t randk_device_workspace(int64_t n, int64_t d);

size_t sel_workspace(const flc_codec_params* prm, int64_t n, int64_t d) {
    size_t b = 0;
    carve_sel(nullptr, prm->codec, n, d, prm->k, &b);
    // RandK: the pattern (compat lists or device draws) is not known at the size query; device
    // draws use the same lists plus the count tree
    if (prm->codec == FLC_RANDK) b += randk_device_workspace(n, d);
    return b;
}

static int grid_stride_blocks(int64_t items, int64_t cap = 4096) {
    return (int)std::max<int64_t>(1, std::min<int64_t>(items, cap));
}

// Runs the TopK / RandK pipeline for n rows and writes out (ASSIGN: n == 1 dense encode).
static int accum_parts() {
    static const int p = [] {
        const char* e = tuning_env("FLC_ACCUM_PARTS");   // tuning runs only (0 / unset: by chunk count)
        const int v = e ? atoi(e) : 0;
        return (v == 1 || v == 2 || v == 4) ? v : 0;
    }();
    return p;
}

static bool assign_fold() {          // tuning runs: FLC_ASSIGN_FOLD=1 writes a lone row's output chunk by chunk
    static const bool v = [] { const char* e = tuning_env("FLC_ASSIGN_FOLD"); return e && atoi(e) == 1; }();
    return v;
}

static bool cs_single() {            // tuning runs: FLC_CS_SINGLE=1 keeps the one-workgroup select for few rows
    static const bool v = [] { const char* e = tuning_env("FLC_CS_SINGLE"); return e && atoi(e) == 1; }();
    return v;
}

#ifndef FLC_LONE_PATH
#define FLC_LONE_PATH 2                // a lone compressVector row: 2 in registers (k_lone_resident, rows up to
#endif                                 // RS_U * 4096 per CU; longer: the list path), 0 the list path
#ifndef FLC_RS_EVREC
#define FLC_RS_EVREC 1                 // the completion event recorded after every resident launch (0: at a stream switch)
#endif
#ifndef FLC_RS_COOP
#define FLC_RS_COOP 0                  // 1: k_lone_resident launched cooperatively (HIP's launch: +22 us a call
#endif                                 // measured; residency holds anyway: G <= CUs, one workgroup per CU, launches serialised)
// k_lone_resident's control block (library-owned, one per device, zeroed once: the kernel leaves it
// clean) and the serialisation of its launches: two resident grids at once could each hold part of
// the chip and wait for the other forever, so a launch on another stream than the previous one
// waits for that one's completion event (one stream: stream order alone)
struct RsCtx {
    uint32_t* ctl = nullptr;
    uint32_t seq = 0;                   // launches so far (tags the tie counts of each call)
    uint32_t xcum = 0;                  // workgroups launched so far (the RS_XGRP counters' sum before a launch)
    hipStream_t last = nullptr;
    hipEvent_t done = nullptr;
};
static std::mutex g_rs_mu;
static std::map<int, RsCtx> g_rs_ctx;
// test hook (flc_debug_resident): the grid of the next resident launches x mult (workgroups that
// cannot all be resident: the abort + repair path, deterministically) and the waits' give-up time
static std::atomic<int> g_rs_dbg_mult{1};
static std::atomic<long long> g_rs_dbg_spin{0};
int rs_debug(int mult, int64_t spin_ticks) {
    if (mult < 1 || mult > 64 || spin_ticks < 0) { set_error("flc_debug_resident: mult 1..64, spin >= 0"); return FLC_ERR_ARG; }
    g_rs_dbg_mult.store(mult);
    g_rs_dbg_spin.store((long long)spin_ticks);
    return FLC_OK;
}
static int rs_cus() {              // compute units of the current device (one k_lone_resident workgroup each)
    static int cu[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    if (!cu[dev]) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
        cu[dev] = c;
    }
    return cu[dev];
}
static int lone_path() {           // tuning runs: env FLC_LONE_PATH overrides
    static const int v = [] { const char* e = tuning_env("FLC_LONE_PATH"); return e ? atoi(e) : FLC_LONE_PATH; }();
    return v;
}

static int filter_group() {
    static const int g = [] {
        const char* e = tuning_env("FLC_FILTER_GS");     // tuning runs only
        return (e && atoi(e) == 2) ? 2 : 4;
    }();
    return g;
}

template <int FGS>
static void launch_filter(RowSrc rows, int64_t n, int64_t r0, int64_t rn, int64_t d, SelWs ws, hipStream_t st,
                          int shards, float* zout = nullptr) {
    // oversubscribed grid (measured: 16-32 K blocks beat a resident-only persistent grid by ~5 %,
    // the hardware dispatcher balances the tail)
    const int64_t waves = rn * ((nchunks(d) + FGS - 1) / FGS);
    const int gw = (int)std::max<int64_t>(1, std::min<int64_t>((waves + 3) / 4, 32768));
    static const int64_t rb = [] {
        // rows per block of the item order: 64 measured 0.5 % faster than row-major (1) at C3
        const char* e = tuning_env("FLC_TK_RB");          // tuning runs only
        return e ? std::max<int64_t>(1, atoll(e)) : (int64_t)64;
    }();
    ProfScope _pv(FGS == 4 ? "k_topk_filter_g4" : "k_topk_filter_g2", st);   // which variant ran (tests)
    if (zout)
        hipLaunchKernelGGL((k_topk_filter_fast<FLC_TK_RING, FGS, 1>), dim3(gw), dim3(256), 0, st, rows, n, r0, rn,
                           std::min(rb, std::max<int64_t>(rn, 1)), d, ws, shards, zout);
    else
        hipLaunchKernelGGL((k_topk_filter_fast<FLC_TK_RING, FGS>), dim3(gw), dim3(256), 0, st, rows, n, r0, rn,
                           std::min(rb, std::max<int64_t>(rn, 1)), d, ws, shards, (float*)nullptr);
}

#ifndef FLC_TK_SPLIT_SAMPLE
#define FLC_TK_SPLIT_SAMPLE 1         // TopK row groups: only group 0's sample before the first filter
#endif
#ifndef FLC_TK_LASTPCT
#define FLC_TK_LASTPCT 100            // size of the last TopK row group in % of the others (its tail is exposed)
#endif
static_assert(FLC_TK_LASTPCT >= 1 && FLC_TK_LASTPCT <= 100, "FLC_TK_LASTPCT: the last row group is 1..100 % of the others");
#ifndef FLC_TK_LAST_TS
#define FLC_TK_LAST_TS 4096           // the exposed last group fold's tile (columns per wave)
#endif
#ifndef FLC_TK_GFOLD
#define FLC_TK_GFOLD 1                // many-row TopK: fold each row group under the next group's filter
#endif
#ifndef FLC_TK_SIDE_NT
#define FLC_TK_SIDE_NT 512            // threads of the side-stream candidate selects (256 or 512)
#endif
#ifndef FLC_TK_EXACT_WG
#define FLC_TK_EXACT_WG 256           // workgroups of the one exact-rows launch (one per CU)
#endif
// Row groups of the TopK fast path whose candidate select + exact fallback run on a side stream
// under the next group's filter (one fold of all rows at the end), at least 64 rows each: 4
// (measured at C3, same box, two runs each: 8.18 ms / step with 1 group, 8.15 with 2, 8.00-8.01
// with 4, 8.04 with 8; profiles/r03/ab_tailov.txt); tuning builds FLC_TK_TAILOV=g.  (The same
// overlap of the sparse QSGD norm + resolve lost at C4, 10.20 -> 10.27-10.44 ms: its filter split
// in groups runs slower; it stays a tuning knob there, FLC_DS_TAILOV.)
static int tk_tail_groups(const flc_codec_params* prm, int64_t n) {
    static const int g = [] { const char* e = tuning_env("FLC_TK_TAILOV"); return e ? std::max(1, atoi(e)) : 4; }();
    const int hint = (prm->flags >> 8) & 0xFF;                       // FLC_ROW_GROUPS(g): the caller's
    if (hint) return (int)std::max<int64_t>(1, std::min<int64_t>(hint, n));
    return (int)std::max<int64_t>(1, std::min<int64_t>(g, n / 64));
}
namespace {
struct TkCtx {
    hipStream_t side = nullptr;
    std::vector<hipEvent_t> ev;
};
std::mutex g_tk_mu;
std::map<int, TkCtx> g_tk_ctx;
}  // namespace

static int launch_chunk_accum(int64_t n, int64_t d, SelWs ws, bool assign, const float* w, float wt, float* out,
                              hipStream_t st);

static RkdWs carve_rkd(void* base, int64_t n, int64_t d, size_t* bytes) {
    Carver cv(base);
    const int64_t C = std::max<int64_t>(host_chunks(d), 1), nn = std::max<int64_t>(n, 1);
    RkdWs s;
    s.cnt = cv.take<uint32_t>((size_t)C * nn);
    s.ckey = cv.take<uint64_t>((size_t)nn);
    if (bytes) *bytes = cv.bytes();
    return s;
}

size_t randk_device_workspace(int64_t n, int64_t d) {
    size_t b = 0;
    carve_rkd(nullptr, n, d, &b);
    return b;
}

static int randk_counts(const flc_codec_params* prm, const flc_pattern* pat, int64_t n, int64_t d, RkdWs ws,
                        hipStream_t st) {
    ProfScope _ps("k_randk_counts", st);
    const int64_t parts = (host_chunks(d) + RKC_BINS - 1) / RKC_BINS;
    hipLaunchKernelGGL(k_randk_counts, dim3((unsigned)parts, (unsigned)n), dim3(RKC_NT), 0, st, n, d, prm->k, prm->seed,
                       pat ? pat->client0 : (int64_t)0, ws);
    FLC_CHECK_LAUNCH("k_randk_counts");
    return FLC_OK;
}

// the device sampler's chunk counts of n clients (flc_device_randk_counts: the sampler's test hook)
int randk_device_counts(uint64_t seed, int64_t client0, int64_t n, int64_t d, int64_t k, uint32_t* cnt, void* wsp,
                        size_t ws_bytes, hipStream_t st) {
    if (ws_bytes < randk_device_workspace(n, d)) { set_error("randk counts: workspace too small"); return FLC_ERR_WORKSPACE; }
    RkdWs ws = carve_rkd(wsp, n, d, nullptr);
    ws.cnt = cnt;                                    // the counts straight into the caller's array
    flc_codec_params prm{};
    prm.codec = FLC_RANDK;
    prm.k = k;
    prm.seed = seed;
    flc_pattern pat{};
    pat.client0 = client0;
    return randk_counts(&prm, &pat, n, d, ws, st);
}

// device-RNG RandK encode + reduce: counts, then the list-free chunk fold
int randk_device_run(const flc_codec_params* prm, const flc_pattern* pat, RowSrc rows, int64_t n, int64_t d,
                     const float* w, float wt, float* out, void* wsp, size_t ws_bytes, hipStream_t st) {
    size_t lb = 0;
    carve_sel(nullptr, FLC_RANDK, n, d, prm->k, &lb);
    if (ws_bytes < lb + randk_device_workspace(n, d)) { set_error("randk: workspace too small"); return FLC_ERR_WORKSPACE; }
    SelWs sw = carve_sel(wsp, FLC_RANDK, n, d, prm->k, nullptr);
    RkdWs rw = carve_rkd(static_cast<char*>(wsp) + lb, n, d, nullptr);
    const int64_t C = host_chunks(d);
    // Long rows (>= 1024 chunks, one wave per chunk fills the chip): the list-free chunk fold, each
    // wave regenerating the rows' members of its chunk.  Short rows: too few chunks for the
    // row-serial fold, so the members are written per row (k_randk_gen) and the chunk fold runs
    // over the lists with its column split (k_chunk_accum).
    // chunk counts: the caller's (flc_pattern.d_randk_counts, made by flc_device_randk_counts) or
    // computed here; the client keys are cheap and always computed here
    auto counts = [&]() -> int {
        if (pat && pat->d_randk_counts) {
            rw.cnt = const_cast<uint32_t*>(pat->d_randk_counts);          // read only below
            hipLaunchKernelGGL(k_randk_ckeys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n, prm->seed,
                               pat->client0, rw.ckey);
            FLC_CHECK_LAUNCH("k_randk_ckeys");
            return FLC_OK;
        }
        return randk_counts(prm, pat, n, d, rw, st);
    };
    if (C >= 1024) {
        if (int rc = counts()) return rc;
        ProfScope _ps("k_randk_fold", st);
        const int ab = grid_stride_blocks((C + 3) / 4, 16384);
        hipLaunchKernelGGL((k_randk_fold<CHUNK>), dim3(ab), dim3(256), 0, st, rows, n, d, rw.cnt, rw.ckey,
                           prm->randk_scale, w, wt, out);
        FLC_CHECK_LAUNCH("k_randk_fold");
        return FLC_OK;
    }
    if (int rc = counts()) return rc;
    hipLaunchKernelGGL(k_randk_tab, dim3((unsigned)n), dim3(256), 0, st, n, d, prm->k, rw.cnt, sw);
    FLC_CHECK_LAUNCH("k_randk_tab");
    {
        ProfScope _ps("k_randk_gen", st);
        const int64_t gx = std::max<int64_t>(1, std::min<int64_t>((C + 4 * RKG_CPW - 1) / (4 * RKG_CPW), 4096));
        hipLaunchKernelGGL(k_randk_gen, dim3((unsigned)gx, (unsigned)std::min<int64_t>(n, 65535)), dim3(256), 0, st, rows,
                           n, d, rw.ckey, prm->randk_scale, sw);
        FLC_CHECK_LAUNCH("k_randk_gen");
    }
    return launch_chunk_accum(n, d, sw, false, w, wt, out, st);
}

// TopK row-group fold: rows [r0, r1) into the running tiles (ws.part); beside a filter the
// one-wave workgroups (<= 102 VGPRs, 16 KB of LDS: room is left beside the filter's waves), the
// exposed last group in 4-wave workgroups
static int launch_group_fold(int64_t n, int64_t d, SelWs ws, const float* w, float wt, float* out, int64_t r0, int64_t r1,
                             bool first, bool last, bool exposed, hipStream_t st) {
    const int64_t C = host_chunks(d);
    ProfScope _ps("k_chunk_accum", st);
    if (!exposed) {
        const int ab = grid_stride_blocks(C, 16384);
        if (w) hipLaunchKernelGGL((k_chunk_accum1<true>), dim3(ab), dim3(64), CHUNK * sizeof(float), st, n, d, ws, w, wt, out, r0, r1,
                                  first ? 1 : 0, last ? 1 : 0);
        else hipLaunchKernelGGL((k_chunk_accum1<false>), dim3(ab), dim3(64), CHUNK * sizeof(float), st, n, d, ws, w, wt, out, r0, r1,
                                first ? 1 : 0, last ? 1 : 0);
    } else {
        constexpr int LTS = FLC_TK_LAST_TS;
        const int ab = grid_stride_blocks((C * (CHUNK / LTS) + 3) / 4, 4096);
        if (w) hipLaunchKernelGGL((k_chunk_accum<false, LTS, true>), dim3(ab), dim3(256), 0, st, n, d, ws, w, wt, out, r0, r1,
                                  first ? 1 : 0, last ? 1 : 0);
        else hipLaunchKernelGGL((k_chunk_accum<false, LTS, false>), dim3(ab), dim3(256), 0, st, n, d, ws, w, wt, out, r0, r1,
                                first ? 1 : 0, last ? 1 : 0);
    }
    FLC_CHECK_LAUNCH("k_chunk_accum(group)");
    return FLC_OK;
}

// chunk-owner fold of the rows' lists (TopK candidates, RandK members)
static int launch_chunk_accum(int64_t n, int64_t d, SelWs ws, bool assign, const float* w, float wt, float* out,
                              hipStream_t st) {
    const int64_t C = host_chunks(d);
    { ProfScope _ps("k_chunk_accum", st);
    // few chunks (short rows: C2's D = 1 M has 245): split each chunk's columns over 2 or 4 waves so
    // the latency-bound row walk runs on more of the chip (many chunks: one wave each, measured best)
    int parts = accum_parts();
    if (parts == 0) parts = C >= 1024 ? 1 : (C >= 256 ? 2 : 4);
    auto go = [&](auto ts, int ab) {
        constexpr int TS = decltype(ts)::value;
        if (assign) hipLaunchKernelGGL((k_chunk_accum<true, TS>), dim3(ab), dim3(256), 0, st, n, d, ws, w, wt, out);
        else if (w) hipLaunchKernelGGL((k_chunk_accum<false, TS, true>), dim3(ab), dim3(256), 0, st, n, d, ws, w, wt, out);
        else hipLaunchKernelGGL((k_chunk_accum<false, TS, false>), dim3(ab), dim3(256), 0, st, n, d, ws, w, wt, out);
    };
    if (parts == 4) go(std::integral_constant<int, CHUNK / 4>{}, grid_stride_blocks((4 * C + 3) / 4, 8192));
    else if (parts == 2) go(std::integral_constant<int, CHUNK / 2>{}, grid_stride_blocks((2 * C + 3) / 4, 8192));
    else if (FLC_CA_WPB1 && !assign) {
        // one-wave workgroups (the tile alone in LDS), one per chunk
        const int ab = grid_stride_blocks(C, 16384);
        if (w) hipLaunchKernelGGL((k_chunk_accum1<true>), dim3(ab), dim3(64), CHUNK * sizeof(float), st, n, d, ws, w, wt, out, (int64_t)0, n, 1, 1);
        else hipLaunchKernelGGL((k_chunk_accum1<false>), dim3(ab), dim3(64), CHUNK * sizeof(float), st, n, d, ws, w, wt, out, (int64_t)0, n, 1, 1);
    } else go(std::integral_constant<int, CHUNK>{}, grid_stride_blocks((C + 3) / 4, 4096));
    }
    FLC_CHECK_LAUNCH("k_chunk_accum");
    return FLC_OK;
}

int sel_run(const flc_codec_params* prm, const flc_pattern* pat, RowSrc rows, bool vec, int64_t n, int64_t d,
            bool assign, const float* w, float wt, float* out, void* wsp, size_t ws_bytes, hipStream_t st) {
    const int codec = prm->codec;
    const int64_t K = prm->k;
    if (d == 0) return FLC_OK;
    if (n == 0) { FLC_CHECK_HIP(hipMemsetAsync(out, 0, (size_t)d * sizeof(float), st)); return FLC_OK; }
    if (K < 1 || K > d) { set_error("K=%lld outside [1, D=%lld]", (long long)K, (long long)d); return FLC_ERR_ARG; }
    if (d >= (int64_t)0xFFFFFFFF) { set_error("D too large for 32-bit entry indices"); return FLC_ERR_ARG; }
    if (codec == FLC_RANDK && !(pat && pat->d_randk_idx))
        return randk_device_run(prm, pat, rows, n, d, w, wt, out, wsp, ws_bytes, st);
    size_t need = 0;
    carve_sel(nullptr, codec, n, d, K, &need);
    if (ws_bytes < need) { set_error("select: workspace %zu < %zu", ws_bytes, need); return FLC_ERR_WORKSPACE; }
    SelWs ws = carve_sel(wsp, codec, n, d, K, nullptr);
    if (codec == FLC_TOPK) {
        if (prm->tie != FLC_TIE_LOWEST && prm->tie != FLC_TIE_HIGHEST) { set_error("topk: unknown tie rule %d", prm->tie); return FLC_ERR_ARG; }
        ws.tie_hi = prm->tie == FLC_TIE_HIGHEST ? 1u : 0u;
    }
    const int64_t C = host_chunks(d);
    bool lone_assign = false, gfold = false;
    // TopK, few rows: sharded candidate lists (k_topk_filter_fast) and the spread select (k_cs_pass)
    const bool few = codec == FLC_TOPK && n <= CS_FEW && !cs_single() && sel_capacity(codec, d, K) >= (int64_t)CS_SH * GCAP;
    if (codec == FLC_RANDK) {
        const int64_t ldi = pat->idx_ld ? pat->idx_ld : K;
        const int64_t spc = rk_spc(C), sb = (C + spc - 1) / spc;
        { ProfScope _ps("k_randk_coarse", st);
        if (spc == 1)
            hipLaunchKernelGGL(k_randk_coarse<true>, dim3((unsigned)n), dim3(RK_T), 0, st, rows, n, d, K, *pat, ldi,
                               prm->randk_scale, ws);
        else
            hipLaunchKernelGGL(k_randk_coarse<false>, dim3((unsigned)n), dim3(RK_T), 0, st, rows, n, d, K, *pat, ldi,
                               prm->randk_scale, ws); }
        FLC_CHECK_LAUNCH("k_randk_coarse");
        if (spc > 1) {
            ProfScope _ps("k_randk_fine", st);
            hipLaunchKernelGGL(k_randk_fine, dim3((unsigned)sb, (unsigned)n), dim3(RK_FTHR), (size_t)spc * sizeof(uint32_t),
                               st, rows, n, d, K, prm->randk_scale, ws);
            FLC_CHECK_LAUNCH("k_randk_fine");
        }
    } else {  // TOPK
        // a lone compressVector row up to RS_U * 4096 elements per CU (any K): in registers, one
        // launch.  Not inside a stream capture (the call's sequence number and the cross-stream
        // serialisation are host state a replayed graph would not redo): the list path there.
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        if (assign && n == 1 && !assign_fold() && lone_path() == 2) FLC_CHECK_HIP(hipStreamIsCapturing(st, &cap));
        if (assign && n == 1 && !assign_fold() && lone_path() == 2 && cap == hipStreamCaptureStatusNone) {
            const int64_t cus = rs_cus();
            const int mult = std::max(1, g_rs_dbg_mult.load());              // (test hook: > 1 forces an aborted call)
            const int64_t G = std::min<int64_t>(cus * mult, (d + RS_NT * 4 - 1) / (RS_NT * 4));
            const int64_t e4 = G > 0 ? (d + G * RS_NT * 4 - 1) / (G * RS_NT * 4) : RS_U + 1;
            if (e4 <= RS_U && d * 4 < ((int64_t)1 << 31)) {
                const int64_t Gu = (d + e4 * RS_NT * 4 - 1) / (e4 * RS_NT * 4);   // no workgroup of padding only
                const long long dspin = g_rs_dbg_spin.load();
                const uint64_t spin = dspin > 0 ? (uint64_t)dspin : (uint64_t)FLC_RS_SPIN;
                ProfScope _ps("k_lone_resident", st);
                int dev = 0;
                FLC_CHECK_HIP(hipGetDevice(&dev));
                std::lock_guard<std::mutex> lk(g_rs_mu);
                RsCtx& rc = g_rs_ctx[dev];
                if (!rc.ctl) {
                    FLC_CHECK_HIP(hipMalloc(reinterpret_cast<void**>(&rc.ctl), (size_t)RS_CTL * sizeof(uint32_t)));
                    FLC_CHECK_HIP(hipMemsetAsync(rc.ctl, 0, (size_t)RS_CTL * sizeof(uint32_t), st));
                    FLC_CHECK_HIP(hipEventCreateWithFlags(&rc.done, FLC_SYNC_EVENT_FLAGS));
                }
                if (rc.last && rc.last != st) {
                    if (!FLC_RS_EVREC) FLC_CHECK_HIP(hipEventRecord(rc.done, rc.last));   // (probe builds)
                    FLC_CHECK_HIP(hipStreamWaitEvent(st, rc.done, 0));
                }
                if (++rc.seq == 0u) rc.seq = 1u;                              // (0: no call; RS_GAVE's cleared value)
                const int e4i = (int)e4;
                if (FLC_RS_COOP) {
                    RowSrc ra = rows;
                    int64_t da = d, ka = K;
                    SelWs wa = ws;
                    float* oa = out;
                    int ea = e4i;
                    uint32_t* ca = rc.ctl;
                    uint32_t sa = rc.seq;
                    uint64_t pa = spin;
                    uint32_t xa = rc.xcum;
                    void* args[] = {&ra, &da, &ka, &wa, &oa, &ea, &ca, &sa, &pa, &xa};
                    FLC_CHECK_HIP(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(&k_lone_resident<RS_U>), dim3((unsigned)Gu),
                                                             dim3(RS_NT), args, 0, st));
                } else {
                    hipLaunchKernelGGL((k_lone_resident<RS_U>), dim3((unsigned)Gu), dim3(RS_NT), 0, st, rows, d, K, ws, out, e4i,
                                       rc.ctl, rc.seq, spin, rc.xcum);
                }
                FLC_CHECK_LAUNCH("k_lone_resident");
                rc.xcum += (uint32_t)Gu;                                      // (every workgroup counts out once)
                if (FLC_RS_EVREC) FLC_CHECK_HIP(hipEventRecord(rc.done, st));
                rc.last = st;
                return FLC_OK;
            }
        }
        const bool dense_k = K * 16 > d;   // large K: the candidate list would not be smaller than the row
        // a lone compressVector (assign, one row) on the fast path: output zeros from the filter, the
        // exact fallback and the scatter in one launch (k_assign_finish)
        lone_assign = assign && n == 1 && few && !dense_k && !assign_fold();

        if (dense_k) FLC_CHECK_HIP(hipMemsetAsync(ws.hist, 0, (size_t)n * HBINS * sizeof(uint32_t), st));
        const int64_t bpr = (C + 3) / 4;
        if (!dense_k) {
            // per row group: filter (the full read), then the candidate select and the exact
            // fallback of the group's rows; with TG > 1 groups the select + fallback of group g run
            // on a side stream under the filter of group g + 1 (both per-row, other rows' lists)
            const int TG = few ? 1 : tk_tail_groups(prm, n);
            // many rows: each group's select does its own exact fallback and its rows are folded
            // right after it (tiles carried in ws.part), under the next group's filter
            gfold = FLC_TK_GFOLD && !few && !assign && !dense_k;
            hipStream_t sside = st;
            TkCtx* cx = nullptr;
            std::unique_lock<std::mutex> lk;
            if (TG > 1) {
                int dev = 0;
                FLC_CHECK_HIP(hipGetDevice(&dev));
                lk = std::unique_lock<std::mutex>(g_tk_mu);
                cx = &g_tk_ctx[dev];
                if (!cx->side) {
                    int lo = 0, hi = 0;
                    FLC_CHECK_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
                    FLC_CHECK_HIP(hipStreamCreateWithPriority(&cx->side, hipStreamNonBlocking, hi));
                }
                while ((int)cx->ev.size() < TG + 3) {
                    hipEvent_t e;
                    FLC_CHECK_HIP(hipEventCreateWithFlags(&e, FLC_SYNC_EVENT_FLAGS));
                    cx->ev.push_back(e);
                }
                sside = cx->side;
            }
            // the sample: group 0's rows before its filter; with row groups the other rows' samples run
            // on the side stream beside group 0's filter (after the work queued before this call), and
            // group 1's filter waits for them — only group 0's share of the sample is exposed
            const bool split = FLC_TK_SPLIT_SAMPLE && TG > 1;
            const int64_t rs1 = split ? group_row(n, TG, 1, FLC_TK_LASTPCT) : n;
            auto sample = [&](int64_t a, int64_t b, hipStream_t sx) {
                if (b <= a) return;
                ProfScope _ps("k_topk_sample", sx);
                // 1024-thread workgroups for any row count (measured 0.098 -> 0.066 ms against 256 at C3)
                hipLaunchKernelGGL((few ? k_topk_sample<1024, true> : k_topk_sample<1024, false>), dim3((unsigned)(b - a)), dim3(1024), 0, sx,
                                   rows, n, d, K, ws, few ? 1 : 0, a);
            };
            if (split) {
                FLC_CHECK_HIP(hipEventRecord(cx->ev[TG + 1], st));
                FLC_CHECK_HIP(hipStreamWaitEvent(sside, cx->ev[TG + 1], 0));
            }
            sample(0, rs1, st);
            FLC_CHECK_LAUNCH("k_topk_sample");
            if (split) {
                sample(rs1, n, sside);
                FLC_CHECK_LAUNCH("k_topk_sample (side)");
                FLC_CHECK_HIP(hipEventRecord(cx->ev[TG + 2], sside));
            }
            for (int g = 0; g < TG; ++g) {
                const int64_t r0 = group_row(n, TG, g, FLC_TK_LASTPCT), rn = group_row(n, TG, g + 1, FLC_TK_LASTPCT) - r0;
                if (split && g == 1) FLC_CHECK_HIP(hipStreamWaitEvent(st, cx->ev[TG + 2], 0));
                { ProfScope _ps("k_topk_filter", st);
                // few rows: 2-chunk groups (twice the waves in flight for a lone row)
                // (one-chunk items for a lone 10 M row measured slower: 26 -> 36 us)
                // a lone compressVector row: the filter also writes the dense output's zeros
                float* zout = lone_assign ? out : nullptr;
                if (filter_group() == 2 || n * d < ((int64_t)64 << 20)) launch_filter<2>(rows, n, r0, rn, d, ws, st, few ? CS_SH : 1, zout);
                else launch_filter<4>(rows, n, r0, rn, d, ws, st, few ? CS_SH : 1, zout); }
                FLC_CHECK_LAUNCH("k_topk_filter");
                if (TG > 1) {
                    FLC_CHECK_HIP(hipEventRecord(cx->ev[g], st));
                    FLC_CHECK_HIP(hipStreamWaitEvent(sside, cx->ev[g], 0));
                }
                { ProfScope _ps("k_cand_select", sside);
                // few rows (a lone compressVector): each list over 64 workgroups, one launch per
                // digit (a finished row's workgroups exit at once); with list mode two launches
                // settle a row whose first digit's bin holds <= CS_LCAP entries (~(4 sqrt(ks) + 8)
                // D / 16 K spread over 256-512 bins: up to ~900 at D = 64 M), else 3 cover every
                // shift; many rows: 512-thread workgroups (measured 0.289 -> 0.263 ms against 256 at C3)
                if (few) {
                    const int np = (FLC_CS_LIST && d <= FLC_CS_TWO_MAXD) ? 2 : 3;
                    for (int p = 0; p < np; ++p)
                        hipLaunchKernelGGL(k_cs_pass, dim3((unsigned)CS_SH, (unsigned)n), dim3(CS_NT), 0, st, K, ws,
                                           p == np - 1 ? 1 : 0);
                } else if (gfold) {
                    // the select with the exact fallback in the same workgroup (every row final after
                    // it), then the group's rows folded into the running tiles, both on the side stream
                    // under the next group's filter (the last group's: exposed)
                    const bool big = rn < 128 || g == TG - 1;
                    const int nt = big ? 1024 : FLC_TK_SIDE_NT;
                    const dim3 grid((unsigned)(big ? rn : grid_stride_blocks(rn, 8192)));
                    if (big) {
                        if (vec) hipLaunchKernelGGL((k_cand_select_x<1024, true>), grid, dim3(nt), 0, sside, rows, n, r0, rn, d, K, ws);
                        else hipLaunchKernelGGL((k_cand_select_x<1024, false>), grid, dim3(nt), 0, sside, rows, n, r0, rn, d, K, ws);
                    } else if (FLC_TK_SIDE_NT == 256) {
                        if (vec) hipLaunchKernelGGL((k_cand_select_x<256, true>), grid, dim3(nt), 0, sside, rows, n, r0, rn, d, K, ws);
                        else hipLaunchKernelGGL((k_cand_select_x<256, false>), grid, dim3(nt), 0, sside, rows, n, r0, rn, d, K, ws);
                    } else {
                        if (vec) hipLaunchKernelGGL((k_cand_select_x<512, true>), grid, dim3(nt), 0, sside, rows, n, r0, rn, d, K, ws);
                        else hipLaunchKernelGGL((k_cand_select_x<512, false>), grid, dim3(nt), 0, sside, rows, n, r0, rn, d, K, ws);
                    }
                } else if (rn < 128 || (TG > 1 && g == TG - 1))
                    // few rows, or the last tail group (its select is exposed, nothing runs beside it):
                    // 1024-thread workgroups, twice the loads in flight per row
                    hipLaunchKernelGGL(k_cand_select<1024>, dim3((unsigned)rn), dim3(1024), 0, sside, r0, rn, K, ws);
                else if (FLC_TK_SIDE_NT == 256)
                    // beside the next group's filter: one wave per SIMD (66 VGPRs) fits in the VGPRs the
                    // filter's three waves per SIMD leave free, so the select co-resides with the
                    // filter's blocks instead of displacing one (512-thread selects slowed the filter
                    // they ran beside by ~8 %, round-4 trace)
                    hipLaunchKernelGGL(k_cand_select<256>, dim3(grid_stride_blocks(rn, 8192)), dim3(256), 0, sside, r0, rn, K, ws);
                else hipLaunchKernelGGL(k_cand_select<512>, dim3(grid_stride_blocks(rn, 8192)), dim3(512), 0, sside, r0, rn, K, ws); }
                FLC_CHECK_LAUNCH("k_cand_select");
                if (gfold) {
                    const bool lastg = g == TG - 1;
                    if (int rc = launch_group_fold(n, d, ws, w, wt, out, r0, r0 + rn, g == 0, lastg, lastg || TG == 1, sside))
                        return rc;
                }
            }
            if (!lone_assign && !gfold) {
                // rows the fast path failed (rare): exact selection of every group's failed rows in
                // ONE launch after the last group's select (a workgroup per row, grid-stride, rows
                // that did not fail return at once).  Per-group launches beside the next group's
                // filter held whole CUs (1024-thread workgroups) while doing nothing: the filters
                // beside them ran 40-110 us slower
                ProfScope _ps("k_topk_exact_rows", sside);
                const int eb = grid_stride_blocks(n, FLC_TK_EXACT_WG);
                if (vec) hipLaunchKernelGGL((k_topk_exact_rows<true>), dim3(eb), dim3(EX_NT), 0, sside, rows, n, (int64_t)0, n, d, K, ws);
                else hipLaunchKernelGGL((k_topk_exact_rows<false>), dim3(eb), dim3(EX_NT), 0, sside, rows, n, (int64_t)0, n, d, K, ws);
                FLC_CHECK_LAUNCH("k_topk_exact_rows");
            }
            if (TG > 1) {
                FLC_CHECK_HIP(hipEventRecord(cx->ev[TG], sside));
                FLC_CHECK_HIP(hipStreamWaitEvent(st, cx->ev[TG], 0));
            }
        } else {
            FLC_CHECK_HIP(hipMemsetAsync(ws.flags, 0, (size_t)n * sizeof(uint32_t), st));
        }
        if (dense_k) {
        // dense K: every row takes the exact multi-launch path
        hipLaunchKernelGGL(k_build_worklist, dim3(1), dim3(1024), 0, st, n, K, d, ws, 1);
        FLC_CHECK_LAUNCH("k_build_worklist");
        const int64_t hb = (d + 65535) / 65536;
        for (int p = 0; p < 3; ++p) {
            { ProfScope _ps("k_radix_hist_full", st);
hipLaunchKernelGGL((k_radix_hist<true>), dim3(grid_stride_blocks(n * hb)), dim3(256), 0, st, rows, n, d, p, ws); }
            FLC_CHECK_LAUNCH("k_radix_hist(full)");
            hipLaunchKernelGGL((k_radix_select<true>), dim3(grid_stride_blocks(n, 1024)), dim3(256), 0, st, n, p, K, ws);
            FLC_CHECK_LAUNCH("k_radix_select(full)");
        }
        hipLaunchKernelGGL(k_tie_count, dim3(grid_stride_blocks(n * bpr, 4096)), dim3(256), 0, st, rows, n, d, ws);
        FLC_CHECK_LAUNCH("k_tie_count");
        hipLaunchKernelGGL(k_tie_scan, dim3(grid_stride_blocks(n, 1024)), dim3(256), 0, st, n, d, ws);
        FLC_CHECK_LAUNCH("k_tie_scan");
        int gb = grid_stride_blocks(n * bpr, 8192);
        { ProfScope _ps("k_topk_filter_exact", st);
if (vec) hipLaunchKernelGGL((k_topk_filter<true, true>), dim3(gb), dim3(256), 0, st, rows, n, d, ws);
        else hipLaunchKernelGGL((k_topk_filter<true, false>), dim3(gb), dim3(256), 0, st, rows, n, d, ws); }
        FLC_CHECK_LAUNCH("k_topk_filter(exact)");
        }
    }
    // Every row's list now holds exactly its admitted entries plus, on the fast path, candidates
    // below the exact threshold; k_chunk_accum admits key >= thr.
    if (lone_assign) {
        // output zeros written by the filter; exact fallback (if the row failed) + scatter
        ProfScope _ps("k_assign_finish", st);
        if (vec) hipLaunchKernelGGL((k_assign_finish<true>), dim3(CS_SH), dim3(EX_NT), 0, st, rows, d, K, ws, out);
        else hipLaunchKernelGGL((k_assign_finish<false>), dim3(CS_SH), dim3(EX_NT), 0, st, rows, d, K, ws, out);
        FLC_CHECK_LAUNCH("k_assign_finish");
        return FLC_OK;
    }
    if (gfold) return FLC_OK;                       // the last group's fold wrote out
    if (assign && n == 1 && codec == FLC_TOPK && !assign_fold()) {
        FLC_CHECK_HIP(hipMemsetAsync(out, 0, (size_t)d * sizeof(float), st));
        const int sb = (int)std::max<int64_t>(1, std::min<int64_t>((sel_capacity(codec, d, K) + 255) / 256, 2048));
        hipLaunchKernelGGL(k_assign_scatter, dim3(sb), dim3(256), 0, st, ws, out, few ? 1 : 0);
        FLC_CHECK_LAUNCH("k_assign_scatter");
        return FLC_OK;
    }
    return launch_chunk_accum(n, d, ws, assign, w, wt, out, st);
}

// flc_select_row_flags: the rows' state words the last TopK sel_run left in the workspace
int sel_row_flags(const flc_codec_params* prm, int64_t n, int64_t d, const void* wsp, size_t ws_bytes,
                  uint32_t* flags, hipStream_t st) {
    if (prm->codec != FLC_TOPK) { set_error("flc_select_row_flags: TopK only"); return FLC_ERR_ARG; }
    if (n <= 0 || d <= 0) return FLC_OK;
    size_t need = 0;
    carve_sel(nullptr, prm->codec, n, d, prm->k, &need);
    if (ws_bytes < need) { set_error("flc_select_row_flags: workspace %zu < %zu", ws_bytes, need); return FLC_ERR_WORKSPACE; }
    const SelWs ws = carve_sel(const_cast<void*>(wsp), prm->codec, n, d, prm->k, nullptr);
    FLC_CHECK_HIP(hipMemcpyAsync(flags, ws.flags, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
    return FLC_OK;
}

// ------------------------------------------------------------------------------------------
// Decode + reduce of sparse wire payloads (wire.hip, SPARSE: 16-B header {fmt, count, norm, bad},
// u32 idx[cap], f32 val[cap], ascending idx): the entries are copied into the selection lists,
// each (chunk, row) range is found by binary search, and k_chunk_accum folds them in row order —
// the same fold as flc_encode_reduce, so the result is the same bits.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_unpack_lists(const char* __restrict__ base, int64_t ld,
                                                      const char* const* __restrict__ ptrs, int64_t n, int64_t cap,
                                                      int64_t pcap, SelWs ws) {
    const int64_t row = blockIdx.y;
    const char* p = base ? base + row * ld : ptrs[row];
    const uint32_t cnt = (uint32_t)min<int64_t>(reinterpret_cast<const uint32_t*>(p)[1], min(cap, pcap));
    const uint32_t* pi = reinterpret_cast<const uint32_t*>(p + 16);
    const float* pv = reinterpret_cast<const float*>(p + 16 + ((4 * pcap + 15) & ~int64_t(15)));
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < cnt; e += (int64_t)gridDim.x * 256) {
        ws.ent_idx[row * ws.cap + e] = pi[e];
        ws.ent_val[row * ws.cap + e] = pv[e];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        ws.thr[row] = 0;
        ws.flags[row] = F_EXACT;
        ws.rowcnt[row * RCS] = cnt;
    }
}

__global__ __launch_bounds__(256) void k_unpack_tab(int64_t n, int64_t d, SelWs ws) {
    const int64_t row = blockIdx.y, C = nchunks(d);
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= C) return;
    const uint32_t cnt = ws.rowcnt[row * RCS];
    const uint32_t* idx = ws.ent_idx + row * ws.cap;
    auto lb = [&](uint64_t key) {
        uint32_t lo = 0, hi = cnt;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if ((uint64_t)idx[mid] < key) lo = mid + 1; else hi = mid;
        }
        return lo;
    };
    const uint32_t a = lb((uint64_t)c << CHUNK_SHIFT), b = lb((uint64_t)(c + 1) << CHUNK_SHIFT);
    ws.tab[c * n + row] = make_uint2(a, b - a);
}

size_t sel_unpack_workspace(const flc_codec_params* prm, int64_t n, int64_t d) {
    size_t b = 0;
    carve_sel(nullptr, FLC_RANDK, n, d, std::max<int64_t>(1, std::min(prm->k, d)), &b);
    return b;
}

int sel_unpack_reduce(const flc_codec_params* prm, const void* base, int64_t ld_bytes, const void* const* ptrs,
                      int64_t n, int64_t d, const float* w, float wt, float* out, void* wsp, size_t ws_bytes,
                      hipStream_t st) {
    const int64_t K = std::max<int64_t>(1, std::min(prm->k, d));
    if (ws_bytes < sel_unpack_workspace(prm, n, d)) { set_error("flc_unpack_reduce: workspace too small"); return FLC_ERR_WORKSPACE; }
    if (d >= (int64_t)0xFFFFFFFF) { set_error("D too large for 32-bit entry indices"); return FLC_ERR_ARG; }
    SelWs ws = carve_sel(wsp, FLC_RANDK, n, d, K, nullptr);
    const int64_t C = host_chunks(d);
    dim3 g1((unsigned)std::max<int64_t>(1, std::min<int64_t>((K + 255) / 256, 64)), (unsigned)n);
    hipLaunchKernelGGL(k_unpack_lists, g1, dim3(256), 0, st, (const char*)base, ld_bytes, (const char* const*)ptrs, n,
                       ws.cap, K, ws);
    FLC_CHECK_LAUNCH("k_unpack_lists");
    hipLaunchKernelGGL(k_unpack_tab, dim3((unsigned)((C + 255) / 256), (unsigned)n), dim3(256), 0, st, n, d, ws);
    FLC_CHECK_LAUNCH("k_unpack_tab");
    const int ab = grid_stride_blocks((C + 3) / 4, 4096);
    { ProfScope _ps("k_chunk_accum", st);
    hipLaunchKernelGGL((k_chunk_accum<false>), dim3(ab), dim3(256), 0, st, n, d, ws, w, wt, out); }
    FLC_CHECK_LAUNCH("k_chunk_accum");
    return FLC_OK;
}

// Dense single-vector RandK: out = 0; out[S] = scale * x[S]  (compressors.py:242-243)
__global__ __launch_bounds__(256) void k_randk_dense(const float* __restrict__ x, int64_t K, const int64_t* __restrict__ idx,
                                                     float scale, float* __restrict__ out) {
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < K; t += (int64_t)gridDim.x * 256) {
        const int64_t j = idx[t];
        out[j] = scale * x[j];
    }
}

int randk_dense(const flc_codec_params* prm, const flc_pattern* pat, const float* x, int64_t d, float* out,
                void* wsp, size_t ws_bytes, hipStream_t st) {
    if (d == 0) return FLC_OK;
    if (prm->k < 1 || prm->k > d) { set_error("randk: K outside [1, D]"); return FLC_ERR_ARG; }
    FLC_CHECK_HIP(hipMemsetAsync(out, 0, (size_t)d * sizeof(float), st));
    if (pat && pat->d_randk_idx) {
        int g = (int)std::max<int64_t>(1, std::min<int64_t>((prm->k + 255) / 256, 1024));
        hipLaunchKernelGGL(k_randk_dense, dim3(g), dim3(256), 0, st, x, prm->k, pat->d_randk_idx, prm->randk_scale, out);
        FLC_CHECK_LAUNCH("k_randk_dense");
        return FLC_OK;
    }
    if (ws_bytes < randk_device_workspace(1, d)) { set_error("randk: workspace too small"); return FLC_ERR_WORKSPACE; }
    RkdWs ws = carve_rkd(wsp, 1, d, nullptr);
    if (int rc = randk_counts(prm, pat, 1, d, ws, st)) return rc;
    const int g = grid_stride_blocks((host_chunks(d) + 3) / 4, 4096);
    hipLaunchKernelGGL(k_randk_scatter_dev, dim3(g), dim3(256), 0, st, x, d, ws.cnt, ws.ckey, prm->randk_scale, out);
    FLC_CHECK_LAUNCH("k_randk_scatter_dev");
    return FLC_OK;
}

}  // namespace flc
