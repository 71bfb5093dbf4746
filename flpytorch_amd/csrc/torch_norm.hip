// The fp32 2-norm in torch's CPU reduction order (compressors.py:272 / 303: `torch.norm(x, p=2)` on
// a CPU fp32 tensor), computed EXACTLY as that sequential order rounds, but in parallel.
//
// The order (oracle/torch_norm.c): 8 lane accumulators, lane l taking x[8k + l]^2 in order as a
// fused multiply-add acc = RN(acc + x^2), the lanes summed left to right, the D % 8 tail added in
// order (fused), then RN(sqrt).  Each lane is a chain of D / 8 dependent roundings — 10.4 ms at
// D = 25 M as a chain (k_norm_torch, codecs.hip: ~8 cycles a step).  This file removes the chain.
//
// Why it parallelises.  While a lane's accumulator stays inside one binade [2^e, 2^(e+1)) its
// rounding grid is fixed: u = 2^(e-23) (below 2^-125, subnormals included, u = 2^-149).  With
// acc = A u (A an integer < 2^24 = AMAX) and x^2 = y exact, RN(acc + y) = (A + c) u where, writing
// y / u = Q + R (Q integer, 0 <= R < 1), c = Q + [R > 1/2] — except a tie R = 1/2, which rounds to
// even and so depends on the parity of A + Q.  So every step is a map A -> A + D(A mod 2) given by
// two integers (D0, D1), and maps compose associatively:
//     (D then G)(p) = D(p) + G((p + D(p)) mod 2),
// so the composite of any run of steps is again two integers, and a scan gives A after every step.
// The composite is exact as long as the result stays below AMAX (the accumulator only grows: the
// final value bounds every intermediate one); the first step that would reach AMAX crosses into
// the next binade and is taken as the real fmaf, after which the next grid applies.  Ties, zeros,
// subnormal accumulators and huge steps are all covered by the same rule; a non-finite x or an
// accumulator overflowing to inf is a "huge" step, taken as the real fmaf.
//
// Three launches per call (rows in parallel, each row's lanes in parallel):
//   k_tn_sums  per part of TN_PS steps of every lane: the float64 sum of x^2 (a prediction only)
//   k_tn_maps  per part: the predicted accumulator at the part's start (the float64 prefix); when
//              the part is predicted inside one binade, the composite map of its steps on that
//              binade's grid — else "no map"
//   k_tn_walk  per row, one wave per lane: walks the parts in order with the exact fp32
//              accumulator: a map whose grid is the accumulator's actual grid and whose result
//              stays below AMAX is applied in O(1); any other part (a crossing inside it, a
//              misprediction, no map) is done exactly by the wave: the part's maps composed on the
//              current grid, a wave scan, the first crossing found and taken as fmaf, repeat.
// Correctness never depends on the prediction (it is verified against the actual accumulator).
// Bit-exact against oracle/torch_norm.c and the reference's own norms (tests/test_gpu_norm_torch.py,
// tests/test_gpu_rows_ref.py).
#include "common.hpp"

namespace flc {

constexpr int TN_PS = 4096;                  // steps of each lane per part (32 768 elements)
constexpr int TN_T = 256;                    // threads of k_tn_sums / k_tn_maps
constexpr int32_t TN_AMAX = 1 << 24;         // a binade's integer range [.., 2^24) in its grid
constexpr int32_t TN_BIG = 1 << 30;          // saturated increment: "crosses, take the real step"
constexpr int TN_XB = 1024;                  // steps per block: the walk's unit (a map each)
constexpr int TN_BPP = TN_PS / TN_XB;        // blocks per part (one wave of k_tn_maps each)
constexpr int TN_NOGRID = -1000;             // no predicted grid: the block has no map
constexpr double TN_MARGIN = 2e-4;           // a predicted range this close to a binade edge: no map

struct TnMap {                               // A -> A + d[A & 1] on the grid 2^eu (valid != 0)
    int32_t d0, d1, eu, valid;
};

struct TnWs {
    double* sums;                            // [n][P][8] float64 sums of x^2 per part and lane
    TnMap* maps;                             // [n][8][P * TN_BPP] per block (a lane's contiguous: the walk's window loads)
    float* lane_acc;                         // [n][8] the lanes' final accumulators
    uint32_t* done;                          // [n] lanes finished (zeroed by k_tn_sums)
};

__host__ __device__ inline int64_t tn_parts(int64_t d) { return ((d - d % 8) / 8 + TN_PS - 1) / TN_PS; }

// one step's map on the grid 2^eu: z = x^2 / 2^eu in float64 — exact: x^2 has at most 48
// significant bits and the scaling only moves the exponent (|z| in [2^-450, 2^410]) — then
// Q = floor(z), R = z - Q (exact) against 1/2
__device__ inline void tn_step(float x, int eu, int32_t& d0, int32_t& d1) {
    const double xd = (double)x;
    const double z = ldexp(xd * xd, -eu);
    if (!(z < (double)TN_BIG)) { d0 = d1 = TN_BIG; return; }          // huge, inf or NaN: the real step
    const double qf = floor(z);
    const double rf = z - qf;
    const int32_t q = (int32_t)qf;
    if (rf > 0.5) { d0 = d1 = q + 1; return; }
    if (rf < 0.5) { d0 = d1 = q; return; }
    d0 = q + (q & 1);                                                  // tie: to even (A + Q even)
    d1 = q + ((q + 1) & 1);
}

// (a then b): a's increment, then b's for the parity a leaves (saturating at TN_BIG)
__device__ inline void tn_compose(int32_t a0, int32_t a1, int32_t b0, int32_t b1, int32_t& c0, int32_t& c1) {
    const int64_t x0 = (int64_t)a0 + ((a0 & 1) ? b1 : b0);
    const int64_t x1 = (int64_t)a1 + ((a1 & 1) ? b0 : b1);           // p = 1: (1 + a1) & 1
    c0 = (int32_t)(x0 > TN_BIG ? TN_BIG : x0);
    c1 = (int32_t)(x1 > TN_BIG ? TN_BIG : x1);
}

// the grid of an accumulator value: acc = A 2^eu with A < 2^24 (acc finite, >= 0)
__device__ inline void tn_grid(float acc, int& eu, int32_t& A) {
    const uint32_t b = __float_as_uint(acc);
    const int ex = (int)(b >> 23);
    if (ex <= 1) {                                                     // acc < 2^-125: the grid 2^-149
        eu = -149;                                                     // (subnormals and [2^-126, 2^-125))
        A = (int32_t)(ex ? ((b & 0x7FFFFFu) | 0x800000u) : b);
    } else {
        eu = ex - 150;
        A = (int32_t)((b & 0x7FFFFFu) | 0x800000u);
    }
}
__device__ inline float tn_value(int32_t A, int eu) { return ldexpf((float)A, eu); }   // exact: A < 2^24

// ------------------------------------------------------------------------------------------
// k_tn_sums: per (part, row) the float64 sums of x^2 of the part's steps, per lane (a prediction).
// Thread t takes steps t, t + TN_T, .. of the part: two float4 loads each (the 8 lanes of a step).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(TN_T) void k_tn_sums(const float* __restrict__ base, int64_t ld, int64_t d, TnWs ws) {
    __shared__ double red[TN_T / 64][8];
    const int64_t P = tn_parts(d), p = blockIdx.x, row = blockIdx.y;
    const float* r = base + row * ld;
    const int64_t steps = (d - d % 8) / 8;
    const int64_t k0 = p * TN_PS, k1 = min(k0 + (int64_t)TN_PS, steps);
    double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(r + 8 * k0), (short)0,
                                                      (int)((k1 - k0) * 32), 0x00020000);
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
#pragma unroll 4
    for (int k = threadIdx.x; k < TN_PS; k += TN_T) {
        const u4v a = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)k * 32u, 0, 2);   // past k1: zeros
        const u4v b = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)k * 32u + 16u, 0, 2);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const double va = (double)__uint_as_float(a[e]), vb = (double)__uint_as_float(b[e]);
            s[e] += va * va;
            s[4 + e] += vb * vb;
        }
    }
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        double v = s[l];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][l] = v;
    }
    __syncthreads();
    if (threadIdx.x < 8) {
        double v = 0;
        for (int w = 0; w < TN_T / 64; ++w) v += red[w][threadIdx.x];
        ws.sums[(row * P + p) * 8 + threadIdx.x] = v;
    }
    if (p == 0 && threadIdx.x == 0) ws.done[row] = 0u;                 // (k_tn_walk's last lane finishes the row)
}

// ------------------------------------------------------------------------------------------
// k_tn_maps: per (part, row): the predicted accumulator at the part's start (the float64 prefix of
// the parts before) and end; when both lie well inside one binade, the part's composite map on
// that binade's grid (each thread composes 16 consecutive steps, then an ordered tree of the 256
// partial maps), else no map.
// ------------------------------------------------------------------------------------------
__device__ inline int tn_predict(double a, double b) {
    // the grid of an accumulator predicted in [a, b], with a margin for the fp32 chain's drift from
    // the float64 sums (a misprediction is caught by k_tn_walk; the margin only makes it rare);
    // TN_NOGRID when the range may straddle a binade
    if (!(b == b && b < 0x1p127)) return TN_NOGRID;
    if (b < 0x1p-125 * (1.0 - TN_MARGIN)) return -149;
    if (a < 0x1p-125 * (1.0 + TN_MARGIN)) return TN_NOGRID;
    int e = 0;
    (void)frexp(a, &e);                                                // a = f 2^e, f in [0.5, 1): binade e - 1
    const double lo = ldexp(1.0, e - 1), hi = ldexp(1.0, e);
    return (a >= lo * (1.0 + TN_MARGIN) && b < hi * (1.0 - TN_MARGIN)) ? e - 1 - 23 : TN_NOGRID;
}

// per (part, row): a map per BLOCK of TN_XB steps.  1024 threads, each with 4 consecutive steps
// of every lane in registers (8 loads in flight a thread, read once); block b = threads 256 b ..
// 256 b + 255 (4 waves).  Each lane's grid predicted for the block from the float64 prefix of the
// parts before, the blocks before in this part and the block's own sum; the steps composed on it,
// then ordered: a wave's shuffle tree, then the block's 4 waves in order.
constexpr int TN_MT = 1024;                  // threads of k_tn_maps
constexpr int TN_MS = TN_PS / TN_MT;         // steps a thread (4)
static_assert(TN_XB == (TN_MT / TN_BPP) * TN_MS, "k_tn_maps: a block is 256 threads' steps");

__global__ __launch_bounds__(TN_MT) void k_tn_maps(const float* __restrict__ base, int64_t ld, int64_t d, TnWs ws) {
    // per thread and lane: its steps' float64 sum, then (reused) its composite map — reduced in
    // order by 32 threads (block b, lane l), one LDS column each: no shuffle chains
    __shared__ double cell[TN_MT][8];
    __shared__ double pre[8], bpre[TN_BPP][8], bsum[TN_BPP][8];
    const int64_t P = tn_parts(d), p = blockIdx.x, row = blockIdx.y;
    const int t = threadIdx.x, blk = t / (TN_MT / TN_BPP);
    constexpr int TPB = TN_MT / TN_BPP;                                // threads per block (256)
    const float* r = base + row * ld;
    const int64_t steps = (d - d % 8) / 8;
    const int64_t k0 = p * TN_PS, k1 = min(k0 + (int64_t)TN_PS, steps);
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(r + 8 * k0), (short)0,
                                                      (int)((k1 - k0) * 32), 0x00020000);
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
    u4v va[TN_MS], vb[TN_MS];
#pragma unroll
    for (int i = 0; i < TN_MS; ++i) {                                  // past k1: zeros (identity steps)
        const uint32_t k = (uint32_t)(t * TN_MS + i);
        va[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, k * 32u, 0, 2);
        vb[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, k * 32u + 16u, 0, 2);
    }
    {                                                                  // the parts before (a prediction):
        double s8[8] = {0, 0, 0, 0, 0, 0, 0, 0};                       // one column of LDS per lane
        for (int64_t q = t; q < p; q += TN_MT)
#pragma unroll
            for (int l = 0; l < 8; ++l) s8[l] += ws.sums[(row * P + q) * 8 + l];
#pragma unroll
        for (int l = 0; l < 8; ++l) cell[t][l] = s8[l];
    }
    __syncthreads();
    if (t < 8) {
        double a = 0;
        for (int i = 0; i < TN_MT; ++i) a += cell[i][t];
        pre[t] = a;
    }
    __syncthreads();
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        double v = 0;
#pragma unroll
        for (int i = 0; i < TN_MS; ++i) {
            const double x = (double)__uint_as_float(l < 4 ? va[i][l & 3] : vb[i][l & 3]);
            v += x * x;
        }
        cell[t][l] = v;
    }
    __syncthreads();
    if (t < 8 * TN_BPP) {                                              // block b's sum of lane l
        const int b = t >> 3, l = t & 7;
        double v = 0;
        for (int i = b * TPB; i < (b + 1) * TPB; ++i) v += cell[i][l];
        bsum[b][l] = v;
    }
    __syncthreads();
    if (t < 8) {
        double a = pre[t];
        for (int b = 0; b < TN_BPP; ++b) { bpre[b][t] = a; a += bsum[b][t]; }
    }
    __syncthreads();
    int eu[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) eu[l] = tn_predict(bpre[blk][l], bpre[blk][l] + bsum[blk][l]);
    __syncthreads();                                                   // (cell reused for the maps)
    int2* mc = reinterpret_cast<int2*>(&cell[0][0]);                   // [TN_MT][8]
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        int32_t a0 = 0, a1 = 0;
#pragma unroll
        for (int i = 0; i < TN_MS; ++i) {
            int32_t s0, s1;
            tn_step(__uint_as_float(l < 4 ? va[i][l & 3] : vb[i][l & 3]), eu[l], s0, s1);
            tn_compose(a0, a1, s0, s1, a0, a1);
        }
        mc[t * 8 + l] = make_int2(a0, a1);
    }
    __syncthreads();
    if (t < 8 * TN_BPP) {                                              // block b's map of lane l, in order
        const int b = t >> 3, l = t & 7;
        int32_t a0 = 0, a1 = 0;
        for (int i = b * TPB; i < (b + 1) * TPB; ++i) {
            const int2 m = mc[i * 8 + l];
            tn_compose(a0, a1, m.x, m.y, a0, a1);
        }
        const int e = tn_predict(bpre[b][l], bpre[b][l] + bsum[b][l]);
        ws.maps[(row * 8 + l) * (P * TN_BPP) + p * TN_BPP + b] = TnMap{a0, a1, e, e != TN_NOGRID ? 1 : 0};
    }
}

// ------------------------------------------------------------------------------------------
// k_tn_walk: per row, wave l walks lane l's chain over the parts with the exact accumulator.
// ------------------------------------------------------------------------------------------
constexpr int TN_WPL = TN_XB / 64;          // steps per wave lane in the exact pass over one block

// the exact pass over steps [k0, k1) of lane l (k1 - k0 <= TN_XB), the accumulator uniform in the
// wave: the block's values staged in LDS by the wave (16 loads a lane in flight), then the chain
// itself, fmaf by fmaf, in one lane (4 values a ds_read_b128, 8 reads ahead): ~8 cycles a step
// whatever the crossings (a map scan per crossing cost more: profiles/r06/norm/walk_probe.txt)
__device__ float tn_block_exact(const float* r, int l, int64_t k0, int64_t k1, float acc, float* stage) {
    const int j = threadIdx.x & 63;
    float xv[TN_WPL];
#pragma unroll
    for (int i = 0; i < TN_WPL; ++i) {
        const int64_t k = k0 + (int64_t)i * 64 + j;                   // coalesced over the lanes
        xv[i] = k < k1 ? r[8 * k + l] : 0.f;                           // (0: fmaf(0, 0, a) == a, a >= 0)
    }
#pragma unroll
    for (int i = 0; i < TN_WPL; ++i) stage[i * 64 + j] = xv[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (j == 0) {
        const float4* s4 = reinterpret_cast<const float4*>(stage);
        constexpr int R = 8;
        float4 cur[R];
#pragma unroll
        for (int u = 0; u < R; ++u) cur[u] = s4[u];
        for (int q = 0; q < TN_XB / 4; q += R) {
            float4 nxt[R];
#pragma unroll
            for (int u = 0; u < R; ++u) nxt[u] = s4[(q + R + u) % (TN_XB / 4)];
#pragma unroll
            for (int u = 0; u < R; ++u) {
                acc = fmaf(cur[u].x, cur[u].x, acc);
                acc = fmaf(cur[u].y, cur[u].y, acc);
                acc = fmaf(cur[u].z, cur[u].z, acc);
                acc = fmaf(cur[u].w, cur[u].w, acc);
            }
#pragma unroll
            for (int u = 0; u < R; ++u) cur[u] = nxt[u];
        }
    }
    acc = __shfl(acc, 0, 64);
    __builtin_amdgcn_wave_barrier();                                   // (stage reused by the next block)
    return acc;
}

// per (lane, row): one wave walks lane l's chain over the blocks with the exact accumulator.
// Windows of 64 x 4 blocks (4 consecutive maps a wave lane, composed while they are on the
// accumulator's grid), the composites scanned in order over the lanes: every leading lane whose 4
// maps hold and whose result stays below AMAX is taken at once; then the first lane's blocks one
// by one, and a block that does not hold is done exactly (tn_block_exact).  The last lane of the
// row to finish sums the 8 lanes left to right, adds the tail and takes the square root.
constexpr int TN_G = 4;                      // blocks per wave lane in a window

__global__ __launch_bounds__(64) void k_tn_walk(const float* __restrict__ base, int64_t ld, int64_t d, TnWs ws,
                                                float* __restrict__ out) {
    __shared__ uint32_t last_s;
    __shared__ __attribute__((aligned(16))) float stage[TN_XB];
    const int l = blockIdx.x;
    const int64_t row = blockIdx.y;
    const int j = threadIdx.x;
    const float* r = base + row * ld;
    const int64_t m = d - d % 8, steps = m / 8;
    const int64_t B = tn_parts(d) * TN_BPP, nb = (steps + TN_XB - 1) / TN_XB;
    const TnMap* mp = ws.maps + (row * 8 + l) * B;
    float acc = 0.f;
    int64_t q = 0;                                                    // next block
#ifdef FLC_TN_PRINT
    uint64_t t_ex = 0, t0w = (uint64_t)wall_clock64();
    int n_ex = 0, n_win = 0;
#endif
    while (q < nb) {
        if ((__float_as_uint(acc) & 0x7FFFFFFFu) >= 0x7F800000u) break;   // inf / NaN: finished below
        int eu;
        int32_t A;
        tn_grid(acc, eu, A);
        TnMap w[TN_G];
#pragma unroll
        for (int g = 0; g < TN_G; ++g) {
            const int64_t bq = q + (int64_t)j * TN_G + g;
            w[g] = bq < nb ? mp[bq] : TnMap{0, 0, TN_NOGRID, 0};
        }
        int32_t c0 = 0, c1 = 0;
        int ng = 0;
#pragma unroll
        for (int g = 0; g < TN_G; ++g)
            if (ng == g && w[g].valid && w[g].eu == eu) { tn_compose(c0, c1, w[g].d0, w[g].d1, c0, c1); ++ng; }
        int full = ng == TN_G;
        for (int o = 1; o < 64; o <<= 1) {
            const int32_t p0 = __shfl_up(c0, o, 64), p1 = __shfl_up(c1, o, 64);
            const int pf = __shfl_up(full, o, 64);
            if (j >= o) { tn_compose(p0, p1, c0, c1, c0, c1); full = full && pf; }
        }
        const int32_t end = A + ((A & 1) ? c1 : c0);
        const uint64_t bad = __ballot(!(full && end < TN_AMAX));
        const int jf = bad ? __ffsll((long long)bad) - 1 : 64;        // leading lanes taken whole
#ifdef FLC_TN_PRINT
        ++n_win;
#endif
        if (jf > 0) {
            acc = tn_value(__shfl(end, jf - 1, 64), eu);
            q += (int64_t)jf * TN_G;
            continue;
        }
        // lane 0's blocks one by one (uniform: its maps broadcast)
        int took = 0;
        for (int g = 0; g < TN_G && q < nb; ++g) {
            const int32_t d0 = __shfl(w[g].d0, 0, 64), d1 = __shfl(w[g].d1, 0, 64);
            const int valid = __shfl(w[g].valid, 0, 64), meu = __shfl(w[g].eu, 0, 64);
            const int32_t nx = A + ((A & 1) ? d1 : d0);
            if (!(valid && meu == eu && nx < TN_AMAX)) break;
            A = nx;
            ++q;
            ++took;
        }
        if (took) { acc = tn_value(A, eu); continue; }
#ifdef FLC_TN_PRINT
        const uint64_t tx = (uint64_t)wall_clock64();
        ++n_ex;
#endif
        acc = tn_block_exact(r, l, q * TN_XB, min((q + 1) * TN_XB, steps), acc, stage);   // block q exactly
#ifdef FLC_TN_PRINT
        t_ex += (uint64_t)wall_clock64() - tx;
#endif
        if ((__float_as_uint(acc) & 0x7FFFFFFFu) >= 0x7F800000u) break; // (q: the block it happened in)
        ++q;
    }
    if ((__float_as_uint(acc) & 0x7FFFFFFFu) >= 0x7F800000u) {
        // a non-finite accumulator: fmaf(x, x, inf) stays inf unless some later x is NaN; NaN stays
        // NaN (scanned from the start of the block where it happened: no NaN can precede it there)
        bool nan = acc != acc;
        for (int64_t k = q * TN_XB + j; k < steps && !nan; k += 64) nan = r[8 * k + l] != r[8 * k + l];
        nan = __ballot(nan) != 0ull;
        if (nan) acc = __uint_as_float(0x7FC00000u);
    }
#ifdef FLC_TN_PRINT
    if (j == 0)
        printf("tn lane %d: %d exact blocks, %d windows, exact %llu of %llu ticks (x10ns)\n", l, n_ex, n_win,
               (unsigned long long)t_ex, (unsigned long long)((uint64_t)wall_clock64() - t0w));
#endif
    if (j == 0) {
        ws.lane_acc[row * 8 + l] = acc;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        last_s = __hip_atomic_fetch_add(ws.done + row, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 7u;
        if (last_s) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    if (last_s && j == 0) {
        const float* la = ws.lane_acc + row * 8;
        float tot = __hip_atomic_load(la, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int k = 1; k < 8; ++k) tot = tot + __hip_atomic_load(la + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int64_t k = m; k < d; ++k) tot = fmaf(r[k], r[k], tot);  // buffer[0] + buffer[1] + ..., the tail
        out[row] = (float)sqrt((double)tot);                           // RN(sqrt): exact via double
    }
}

static TnWs carve_tn(void* base, int64_t n, int64_t d, size_t* bytes) {
    Carver cv(base);
    const int64_t P = std::max<int64_t>(tn_parts(d), 1), nn = std::max<int64_t>(n, 1);
    TnWs w;
    w.sums = cv.take<double>((size_t)nn * P * 8);
    w.maps = cv.take<TnMap>((size_t)nn * P * TN_BPP * 8);
    w.lane_acc = cv.take<float>((size_t)nn * 8);
    w.done = cv.take<uint32_t>((size_t)nn);
    if (bytes) *bytes = cv.bytes();
    return w;
}

size_t norm_torch_ws_bytes(int64_t n, int64_t d) {
    size_t b = 0;
    carve_tn(nullptr, n, d, &b);
    return b;
}

int norm_torch_ws_run(const float* x, int64_t ld, int64_t n, int64_t d, float* out, void* wsp, size_t ws_bytes,
                      hipStream_t st) {
    if (n <= 0) return FLC_OK;
    if (ws_bytes < norm_torch_ws_bytes(n, d)) { set_error("flc_norm2_torch_cpu_ws: workspace too small"); return FLC_ERR_WORKSPACE; }
    const TnWs ws = carve_tn(wsp, n, d, nullptr);
    const int64_t P = tn_parts(d);
    if (P > 0) {
        if (n > 65535) { set_error("flc_norm2_torch_cpu_ws: n > 65535"); return FLC_ERR_ARG; }
        { ProfScope _ps("k_tn_sums", st);
        hipLaunchKernelGGL(k_tn_sums, dim3((unsigned)P, (unsigned)n), dim3(TN_T), 0, st, x, ld, d, ws); }
        FLC_CHECK_LAUNCH("k_tn_sums");
        { ProfScope _ps("k_tn_maps", st);
        hipLaunchKernelGGL(k_tn_maps, dim3((unsigned)P, (unsigned)n), dim3(TN_MT), 0, st, x, ld, d, ws); }
        FLC_CHECK_LAUNCH("k_tn_maps");
    }
    if (P == 0) FLC_CHECK_HIP(hipMemsetAsync(ws.done, 0, (size_t)n * sizeof(uint32_t), st));   // (no k_tn_sums)
    { ProfScope _ps("k_tn_walk", st);
    hipLaunchKernelGGL(k_tn_walk, dim3(8u, (unsigned)n), dim3(64), 0, st, x, ld, d, ws, out); }
    FLC_CHECK_LAUNCH("k_tn_walk");
    return FLC_OK;
}

}  // namespace flc
