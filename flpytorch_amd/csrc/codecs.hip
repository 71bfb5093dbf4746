// Elementwise codecs: ident / lazy (Bernoulli) / natural / standard dithering (QSGD, TernGrad) /
// natural dithering — fl_pytorch/utils/compressors.py:227-329 — plus the per-row p-norms.
//
// Two output forms share one per-element codec functor:
//   * dense encode (compressVector): out[j] = C(x)[j]                     (k_ew_dense)
//   * fused encode+reduce:            out[j] = (sum_i w_i C_i(row_i)[j]) / w_total (k_ew_accum)
//     "tile owner": each thread owns COLS float4 column groups in registers and walks the N
//     rows in order, so the fp32 sum is the reference's sequential one, bit for bit.
//
// Exactness notes (all mirrored from the reference's torch-CPU op order):
//   y = |x| / pnorm and p = (y - l[s+1]) / (l[s] - l[s+1]) are IEEE fp32 divisions;
//   the float64 uniform is compared with p promoted to float64 (compressors.py:288);
//   out = (level * sign) * pnorm, left to right (296); natural dithering returns
//   (y * sign) * pnorm (the reference's line 326); natural uses a correctly rounded fp32 log2.
// Norms accumulate in float64 (exactly rounded fp32 result); torch's CPU norm is not
// (see DESIGN.md), so parity is stated against the exactly rounded norm.
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "codec_ops.hpp"
#include "wire_codes.hpp"

namespace flc {

// ------------------------------------------------------------------------------------------
// p-norms: partial[row][part] (float64, fixed slots) then one wave per row folds them in a
// fixed order -> deterministic, exactly rounded fp32 norm.
// ------------------------------------------------------------------------------------------
constexpr int NORM_PART = 65536;   // elements per partial (256 threads x 64 elements) ...
constexpr int NORM_PART_MIN = 4096; // ... halved for few rows so a short launch still spans the chip

// elements per partial for n rows of d: 65536, halved (down to 4096) while n * parts < 2048
int64_t norm_part_len(int64_t n, int64_t d) {
    int64_t len = NORM_PART;
    while (len > NORM_PART_MIN && std::max<int64_t>(n, 1) * ((d + len - 1) / len) < 2048) len >>= 1;
    return len;
}

template <int NORM>
__device__ inline double nacc(double a, float v) {
    if (NORM == FLC_NORM_LINF) { double f = fabs((double)v); return (f > a || f != f) ? f : a; }
    if (NORM == FLC_NORM_L1) return a + fabs((double)v);
    return fma((double)v, (double)v, a);
}
template <int NORM>
__device__ inline double ncomb(double a, double b) {
    if (NORM == FLC_NORM_LINF) return (b > a || b != b) ? b : a;
    return a + b;
}

// nonzero |v| below 2^-80: the row cannot use the unguarded fast division (div_fast)
__device__ inline uint32_t is_tiny(float v) { const float a = fabsf(v); return (a != 0.f && a < 0x1p-80f) ? 1u : 0u; }

// DIFF: the row is the fp32 difference src.row(0) - sub (the shift codecs' C(a - b), one row)
template <int NORM, bool VEC, bool DIFF, bool KEEP = false>
__global__ __launch_bounds__(256) void k_norm_partials(RowSrc src, const float* __restrict__ sub, int64_t d,
                                                       int64_t parts, int64_t plen, double* __restrict__ partial,
                                                       uint32_t* __restrict__ tinyp) {
    const int64_t row = blockIdx.y;
    const float* r = src.row(row);
    auto ld1 = [&](int64_t j) -> float { return DIFF ? r[j] - sub[j] : r[j]; };
    __shared__ double red[4];
    __shared__ uint32_t redt[4];
    for (int64_t part = blockIdx.x; part < parts; part += gridDim.x) {
        const int64_t j0 = part * plen;
        const int64_t j1 = min(d, j0 + plen);
        double a = 0.0;
        uint32_t tiny = 0;
        if (VEC) {
            const int64_t g0 = j0 / 4, g1 = j1 / 4;   // j0 % 4 == 0 (plen % 4 == 0)
            int64_t g = g0 + threadIdx.x;
            if (!DIFF) {
                // 8 loads in flight per thread, accumulated in the same order as one at a time
                for (; g + 7 * 256 < g1; g += 8 * 256) {
                    float4 q[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u)
                        q[u] = KEEP ? reinterpret_cast<const float4*>(r)[g + u * 256] : ld_row4(reinterpret_cast<const float4*>(r) + g + u * 256);
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        a = nacc<NORM>(a, q[u].x); a = nacc<NORM>(a, q[u].y); a = nacc<NORM>(a, q[u].z); a = nacc<NORM>(a, q[u].w);
                        tiny |= is_tiny(q[u].x) | is_tiny(q[u].y) | is_tiny(q[u].z) | is_tiny(q[u].w);
                    }
                }
            }
            for (; g < g1; g += 256) {
                float4 v = ld_row4(reinterpret_cast<const float4*>(r) + g);
                if (DIFF) {
                    const float4 u = reinterpret_cast<const float4*>(sub)[g];
                    v = make_float4(v.x - u.x, v.y - u.y, v.z - u.z, v.w - u.w);
                }
                a = nacc<NORM>(a, v.x); a = nacc<NORM>(a, v.y); a = nacc<NORM>(a, v.z); a = nacc<NORM>(a, v.w);
                tiny |= is_tiny(v.x) | is_tiny(v.y) | is_tiny(v.z) | is_tiny(v.w);
            }
            for (int64_t j = g1 * 4 + threadIdx.x; j < j1; j += 256) { const float v = ld1(j); a = nacc<NORM>(a, v); tiny |= is_tiny(v); }
        } else {
            for (int64_t j = j0 + threadIdx.x; j < j1; j += 256) { const float v = ld1(j); a = nacc<NORM>(a, v); tiny |= is_tiny(v); }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            a = ncomb<NORM>(a, __shfl_xor(a, o, WAVE));
            tiny |= __shfl_xor(tiny, o, WAVE);
        }
        if ((threadIdx.x & 63) == 0) { red[threadIdx.x >> 6] = a; redt[threadIdx.x >> 6] = tiny; }
        __syncthreads();
        if (threadIdx.x == 0) {
            partial[row * parts + part] = ncomb<NORM>(ncomb<NORM>(red[0], red[1]), ncomb<NORM>(red[2], red[3]));
            tinyp[row * parts + part] = redt[0] | redt[1] | redt[2] | redt[3];
        }
        __syncthreads();
    }
}

// Per row: the norm, RN(1/norm), rowfast = 1 when the encode may divide by the norm with the
// unguarded div_fast (norm inside [2^-40, 2^80], no nonzero element below 2^-80), and the
// device-RNG row key.
template <int NORM>
__global__ __launch_bounds__(64) void k_norm_final(const double* __restrict__ partial,
                                                   const uint32_t* __restrict__ tinyp, int64_t parts,
                                                   int64_t n, float* __restrict__ pn, float* __restrict__ rpn,
                                                   uint32_t* __restrict__ rowfast, uint64_t seed, int64_t client0,
                                                   uint32_t* __restrict__ rk) {
    const int64_t row = blockIdx.x;
    if (row >= n) return;
    double a = 0.0;
    uint32_t tiny = 0;
    // lane t combines partials t, t + 64, ... in that order; 8 of them loaded per round trip (the
    // partials come from every XCD: each load is a far miss, thousands of them for a lone row)
    const double* pr = partial + row * parts;
    const uint32_t* tr = tinyp + row * parts;
    int64_t p = threadIdx.x;
    for (; p + 7 * 64 < parts; p += 8 * 64) {
        double v[8];
        uint32_t t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) { v[u] = pr[p + u * 64]; t[u] = tr[p + u * 64]; }
#pragma unroll
        for (int u = 0; u < 8; ++u) { a = ncomb<NORM>(a, v[u]); tiny |= t[u]; }
    }
    for (; p < parts; p += 64) {
        a = ncomb<NORM>(a, pr[p]);
        tiny |= tr[p];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        a = ncomb<NORM>(a, __shfl_xor(a, o, WAVE));
        tiny |= __shfl_xor(tiny, o, WAVE);
    }
    if (threadIdx.x == 0) {
        const float v = (NORM == FLC_NORM_L2) ? (float)sqrt(a) : (float)a;
        pn[row] = v;
        rpn[row] = 1.0f / v;
        rowfast[row] = (!tiny && v >= 0x1p-40f && v <= 0x1p80f) ? 1u : 0u;
        rk[row] = rowkey(client_key(seed, client0 + row));
    }
}

int64_t norm_parts(int64_t n, int64_t d) { const int64_t l = norm_part_len(n, d); return (d + l - 1) / l; }

int launch_norms(RowSrc src, bool vec, int64_t n, int64_t d, int norm, double* partial, uint32_t* tinyp,
                 float* pn, float* rpn, uint32_t* rowfast, uint64_t seed, int64_t client0, uint32_t* rk,
                 hipStream_t st, const float* sub) {
    if (sub && n != 1) { set_error("launch_norms: a difference source is one row"); return FLC_ERR_ARG; }
    const int64_t parts = norm_parts(n, d), plen = norm_part_len(n, d);
    if (n == 0) return FLC_OK;
    if (parts == 0) {  // d == 0: norm of an empty vector
        FLC_CHECK_HIP(hipMemsetAsync(pn, 0, (size_t)n * sizeof(float), st));
        FLC_CHECK_HIP(hipMemsetAsync(rowfast, 0, (size_t)n * sizeof(uint32_t), st));
        FLC_CHECK_HIP(hipMemsetAsync(rk, 0, (size_t)n * sizeof(uint32_t), st));
        return FLC_OK;
    }
    // blocks per row: up to 64 for many rows, more when the rows are few (all parts in flight)
    dim3 grid((unsigned)std::min<int64_t>(parts, std::max<int64_t>(64, 4096 / std::max<int64_t>(n, 1))), (unsigned)n);
#define FLC_NORM_CASE(NK)                                                                           \
    { ProfScope _ps("k_norm_partials", st);                                                         \
    if (sub && vec) hipLaunchKernelGGL((k_norm_partials<NK, true, true>), grid, dim3(256), 0, st, src, sub, d, parts, plen, partial, tinyp); \
    else if (sub) hipLaunchKernelGGL((k_norm_partials<NK, false, true>), grid, dim3(256), 0, st, src, sub, d, parts, plen, partial, tinyp); \
    else if (vec) hipLaunchKernelGGL((k_norm_partials<NK, true, false>), grid, dim3(256), 0, st, src, sub, d, parts, plen, partial, tinyp); \
    else hipLaunchKernelGGL((k_norm_partials<NK, false, false>), grid, dim3(256), 0, st, src, sub, d, parts, plen, partial, tinyp); } \
    FLC_CHECK_LAUNCH("k_norm_partials");                                                            \
    hipLaunchKernelGGL((k_norm_final<NK>), dim3((unsigned)n), dim3(64), 0, st, partial, tinyp, parts, n, pn, rpn,   \
                       rowfast, seed, client0, rk);                                                 \
    FLC_CHECK_LAUNCH("k_norm_final");
    if (norm == FLC_NORM_L2) { FLC_NORM_CASE(FLC_NORM_L2) }
    else if (norm == FLC_NORM_L1) { FLC_NORM_CASE(FLC_NORM_L1) }
    else { FLC_NORM_CASE(FLC_NORM_LINF) }
#undef FLC_NORM_CASE
    return FLC_OK;
}

// ------------------------------------------------------------------------------------------
// Dense encode of one row (compressVector).
// ------------------------------------------------------------------------------------------
template <class Op, bool VEC>
__global__ __launch_bounds__(256) void k_ew_dense(const float* __restrict__ x, int64_t d, Op op,
                                                  const float* __restrict__ levels, int s, float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float4 smem_tab[];
    if (Op::TABLE) op.set_table_ok(load_table(levels, s, smem_tab));
    op.setup(0);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t j0 = VEC ? (d / 4) * 4 : 0;
    if (VEC) {
        for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < d / 4; g += stride) {
            uint32_t cs[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) cs[q] = op.col(g * 4 + q);
            const float4 v = reinterpret_cast<const float4*>(x)[g];
            reinterpret_cast<float4*>(out)[g] = op.row_fast() ? apply4<true>(op, v, g * 4, cs, smem_tab)
                                                              : apply4<false>(op, v, g * 4, cs, smem_tab);
        }
    }
    for (int64_t j = j0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += stride)
        out[j] = op.template apply<false>(x[j], j, op.col(j), smem_tab);
}

// ------------------------------------------------------------------------------------------
// A lone row's standard dithering (compressVector, own norm): after the norm partials, ONE launch
// in which every workgroup folds the partials itself (fixed order: the same norm in every block)
// and encodes U float4 groups per thread per trip with all their loads — the row's and, in compat
// mode, the float64 draws' — issued before the arithmetic.  Replaces k_norm_final + k_ew_dense
// (one launch boundary less; the grid-stride loop of k_ew_dense kept one load per thread in flight).
// ------------------------------------------------------------------------------------------
// 65536-element partials (382 norm workgroups at D = 25 M), 1024 encode workgroups of 2 groups
// per thread per trip: 88.0 -> 82.8 us per call against 32768 / 2048 / 4 (compat, D = 25 M, same
// box; 1024 / 4 / 32768 85.2, 768 or 1536 workgroups 87.5 / 84.1, 131072-element partials 86.8),
// profiles/r04/lone_ab.txt
#ifndef FLC_LONE_PLEN
#define FLC_LONE_PLEN 65536
#endif
#ifndef FLC_LONE_GRID
#define FLC_LONE_GRID 1024
#endif
constexpr int64_t LONE_PLEN = FLC_LONE_PLEN;  // elements per norm partial of a lone row
#ifndef FLC_LONE_U
#define FLC_LONE_U 2
#endif
// The norm pass reads the row with ordinary loads, so the encode's second read of it finds it in
// the caches (the 100 MB row of C4 fits the 256 MB infinity cache), and the encode's output goes
// out with nontemporal stores: 93.5 -> 87.7 us per call at D = 25 M in compat mode (same box,
// interleaved runs; each alone: 90.7 / 93.3 us; 8 groups per trip: 95.7 us), profiles/r04/lone_ab.txt
#ifndef FLC_LONE_KEEP
#define FLC_LONE_KEEP 1
#endif
#ifndef FLC_LONE_OUT_NT
#define FLC_LONE_OUT_NT 1
#endif
constexpr int LONE_U = FLC_LONE_U;            // float4 groups per thread per trip

template <int NORM, bool COMPAT, bool F>
__device__ inline void lone_dither_body(const DitherOp<false, COMPAT>& op, const float* __restrict__ x, int64_t d,
                                        const float4* tab, float* __restrict__ out) {
    const int64_t n4 = d / 4;
    const float4* x4 = reinterpret_cast<const float4*>(x);
    typedef double v2d __attribute__((ext_vector_type(2)));
    for (int64_t b = (int64_t)blockIdx.x * 256 * LONE_U; b < n4; b += (int64_t)gridDim.x * 256 * LONE_U) {
        float4 v[LONE_U];
        double uu[LONE_U][4];
#pragma unroll
        for (int u = 0; u < LONE_U; ++u) {
            const int64_t g = b + u * 256 + threadIdx.x;
            const bool in = g < n4;
            v[u] = in ? (FLC_LONE_KEEP ? x4[g] : ld_row4(x4 + g)) : make_float4(0.f, 0.f, 0.f, 0.f);
            if constexpr (COMPAT) {
                const v2d* up = reinterpret_cast<const v2d*>(op.urow + 4 * g);
                const v2d a = in ? __builtin_nontemporal_load(up) : v2d{0.0, 0.0};
                const v2d c = in ? __builtin_nontemporal_load(up + 1) : v2d{0.0, 0.0};
                uu[u][0] = a.x; uu[u][1] = a.y; uu[u][2] = c.x; uu[u][3] = c.y;
            }
        }
#pragma unroll
        for (int u = 0; u < LONE_U; ++u) {
            const int64_t g = b + u * 256 + threadIdx.x;
            if (g >= n4) continue;
            const float xe[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
            const int64_t jv[4] = {g * 4, g * 4 + 1, g * 4 + 2, g * 4 + 3};
            uint32_t cs[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) cs[q] = op.col(g * 4 + q);
            float o[4];
            op.template apply_block<F, 4>(xe, jv, cs, tab, o, COMPAT ? uu[u] : nullptr);
            if (FLC_LONE_OUT_NT) {
                typedef float v4f __attribute__((ext_vector_type(4)));
                __builtin_nontemporal_store(v4f{o[0], o[1], o[2], o[3]}, reinterpret_cast<v4f*>(out) + g);
            } else {
                reinterpret_cast<float4*>(out)[g] = make_float4(o[0], o[1], o[2], o[3]);
            }
        }
    }
    for (int64_t j = n4 * 4 + (int64_t)blockIdx.x * 256 + threadIdx.x; j < d; j += (int64_t)gridDim.x * 256)
        out[j] = op.template apply<false>(x[j], j, op.col(j), tab);
}

template <int NORM, bool COMPAT>
__global__ __launch_bounds__(256) void k_lone_dither(const float* __restrict__ x, int64_t d, DitherOp<false, COMPAT> op,
                                                     const float* __restrict__ levels, int s, float* __restrict__ out,
                                                     const double* __restrict__ partial, const uint32_t* __restrict__ tinyp,
                                                     int64_t parts, float* __restrict__ pn, float* __restrict__ rpn,
                                                     uint32_t* __restrict__ rowfast, uint64_t seed, int64_t client0,
                                                     uint32_t* __restrict__ rk, float* __restrict__ pout) {
    extern __shared__ __attribute__((aligned(16))) float4 smem_tab[];
    __shared__ double red[4];
    __shared__ uint32_t redt[4];
    const bool tab_ok = load_table(levels, s, smem_tab);
    // the norm: thread t folds partials t, t + 256, ... in order, then the waves' sums in order
    double a = 0.0;
    uint32_t tiny = 0;
    for (int64_t p = threadIdx.x; p < parts; p += 256) { a = ncomb<NORM>(a, partial[p]); tiny |= tinyp[p]; }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        a = ncomb<NORM>(a, __shfl_xor(a, o, WAVE));
        tiny |= __shfl_xor(tiny, o, WAVE);
    }
    if ((threadIdx.x & 63) == 0) { red[threadIdx.x >> 6] = a; redt[threadIdx.x >> 6] = tiny; }
    __syncthreads();
    a = ncomb<NORM>(ncomb<NORM>(ncomb<NORM>(red[0], red[1]), red[2]), red[3]);
    tiny = redt[0] | redt[1] | redt[2] | redt[3];
    const float v = (NORM == FLC_NORM_L2) ? (float)sqrt(a) : (float)a;
    const bool fast = !tiny && v >= 0x1p-40f && v <= 0x1p80f;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        pn[0] = v;
        rpn[0] = 1.0f / v;
        rowfast[0] = fast ? 1u : 0u;
        rk[0] = rowkey(client_key(seed, client0));
        if (pout) pout[0] = v;
    }
    op.dn.b = v;
    op.dn.rb = 1.0f / v;
    op.dn.ok = fabsf(v) >= 0x1p-40f && fabsf(v) <= 0x1p80f;
    op.fast = fast && tab_ok;
    op.tab_ok = tab_ok;
    op.urow = COMPAT ? op.us.u : nullptr;
    op.rk = COMPAT ? 0u : rowkey(client_key(seed, client0));
    if (op.fast) lone_dither_body<NORM, COMPAT, true>(op, x, d, smem_tab, out);
    else lone_dither_body<NORM, COMPAT, false>(op, x, d, smem_tab, out);
}

// ------------------------------------------------------------------------------------------
// Encode straight to wire codes (flc_pack of the Q8 / Q16 / NAT16 formats): the dense value of
// each element is formed exactly as k_ew_dense forms it and turned into its code in registers,
// so the client's message costs one read of the row (plus the norm pass) and one write of codes.
// ------------------------------------------------------------------------------------------
template <class Op, bool VEC>
__global__ __launch_bounds__(256) void k_ew_code(const float* __restrict__ x, int64_t d, Op op,
                                                 const float* __restrict__ levels, int s, CodeArgs ca) {
    extern __shared__ __attribute__((aligned(16))) float4 smem_tab[];
    if (Op::TABLE) op.set_table_ok(load_table(levels, s, smem_tab));
    op.setup(0);
    PayloadHeader* h = reinterpret_cast<PayloadHeader*>(ca.payload);
    char* body = ca.payload + 16;
    const float norm = ca.pn ? *ca.pn : 0.f;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        h->fmt = (uint32_t)ca.fmt;
        h->count = (uint32_t)d;
        h->norm = norm;
    }
    const uint32_t sbit = ca.fmt == FMT_Q8 ? 0x80u : 0x8000u;
    auto code = [&](float v) -> uint32_t {
        return ca.fmt == FMT_NAT16 ? nat_code(v) : lev_code(v, ca.lv, ca.s, norm, sbit, &h->bad);
    };
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t j0 = VEC ? (d / 4) * 4 : 0;
    if (VEC) {
        for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < d / 4; g += stride) {
            uint32_t cs[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) cs[q] = op.col(g * 4 + q);
            const float4 v = reinterpret_cast<const float4*>(x)[g];
            const float4 e = op.row_fast() ? apply4<true>(op, v, g * 4, cs, smem_tab)
                                           : apply4<false>(op, v, g * 4, cs, smem_tab);
            const uint32_t c0 = code(e.x), c1 = code(e.y), c2 = code(e.z), c3 = code(e.w);
            if (ca.fmt == FMT_Q8)
                reinterpret_cast<uint32_t*>(body)[g] = c0 | (c1 << 8) | (c2 << 16) | (c3 << 24);
            else
                reinterpret_cast<uint2*>(body)[g] = make_uint2(c0 | (c1 << 16), c2 | (c3 << 16));
        }
    }
    for (int64_t j = j0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += stride) {
        const uint32_t c = code(op.template apply<false>(x[j], j, op.col(j), smem_tab));
        if (ca.fmt == FMT_Q8) reinterpret_cast<uint8_t*>(body)[j] = (uint8_t)c;
        else reinterpret_cast<uint16_t*>(body)[j] = (uint16_t)c;
    }
}

static int grid_cap(int64_t work, int64_t per_block, int64_t cap);

template <class Op>
static int launch_code(const float* x, int64_t d, Op op, const float* levels, int s, const CodeArgs& ca, hipStream_t st) {
    if (d == 0) return FLC_OK;
    const bool vec = ((uintptr_t)x & 15u) == 0;
    const size_t lds = Op::TABLE ? (size_t)s * sizeof(float4) : 0;
    const int grid = grid_cap(vec ? (d + 3) / 4 : d, 256, 4096);
    if (vec) hipLaunchKernelGGL((k_ew_code<Op, true>), dim3(grid), dim3(256), lds, st, x, d, op, levels, s, ca);
    else hipLaunchKernelGGL((k_ew_code<Op, false>), dim3(grid), dim3(256), lds, st, x, d, op, levels, s, ca);
    FLC_CHECK_LAUNCH("k_ew_code");
    return FLC_OK;
}

// ------------------------------------------------------------------------------------------
// Shift codecs, one row (algorithms.py DIANA 1383-1391, EF21 1506-1517, MARINA
// 537 / 691, FRECON 1104-1110, COFIG 1265-1269): e = C(a - b) is never stored —
//     msg   = base + e * scale   (or e * scale without a base)
//     h_out = h_in + alpha * e
// each op rounded separately in fp32 (torch scalar ops on fp32 tensors take the scalar as fp32).
// Every element is read and written by one thread, so msg / h_out may alias a, b, base or h_in.
// ------------------------------------------------------------------------------------------
__device__ inline void shift_epi1(const ShiftArgs& sh, int64_t j, float e) {
    if (sh.msg) {
        const float t = e * sh.scale;
        sh.msg[j] = sh.base ? sh.base[j] + t : t;
    }
    if (sh.hout) sh.hout[j] = sh.hin[j] + sh.alpha * e;
}

template <class Op, bool VEC>
__global__ __launch_bounds__(256) void k_ew_shift(const float* __restrict__ a, int64_t d, Op op,
                                                  const float* __restrict__ levels, int s, ShiftArgs sh) {
    extern __shared__ __attribute__((aligned(16))) float4 smem_tab[];
    if (Op::TABLE) op.set_table_ok(load_table(levels, s, smem_tab));
    op.setup(0);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t j0 = VEC ? (d / 4) * 4 : 0;
    if (VEC) {
        for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < d / 4; g += stride) {
            uint32_t cs[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) cs[q] = op.col(g * 4 + q);
            const float4 x = reinterpret_cast<const float4*>(a)[g];
            const float4 y = reinterpret_cast<const float4*>(sh.b)[g];
            const float4 v = make_float4(x.x - y.x, x.y - y.y, x.z - y.z, x.w - y.w);
            const float4 e = op.row_fast() ? apply4<true>(op, v, g * 4, cs, smem_tab)
                                           : apply4<false>(op, v, g * 4, cs, smem_tab);
            if (sh.msg) {
                const float4 t = make_float4(e.x * sh.scale, e.y * sh.scale, e.z * sh.scale, e.w * sh.scale);
                float4 m = t;
                if (sh.base) {
                    const float4 bs = reinterpret_cast<const float4*>(sh.base)[g];
                    m = make_float4(bs.x + t.x, bs.y + t.y, bs.z + t.z, bs.w + t.w);
                }
                reinterpret_cast<float4*>(sh.msg)[g] = m;
            }
            if (sh.hout) {
                const float4 h = reinterpret_cast<const float4*>(sh.hin)[g];
                reinterpret_cast<float4*>(sh.hout)[g] =
                    make_float4(h.x + sh.alpha * e.x, h.y + sh.alpha * e.y, h.z + sh.alpha * e.z, h.w + sh.alpha * e.w);
            }
        }
    }
    for (int64_t j = j0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += stride)
        shift_epi1(sh, j, op.template apply<false>(a[j] - sh.b[j], j, op.col(j), smem_tab));
}

// ------------------------------------------------------------------------------------------
// Fused encode + reduce over N rows.  Tile owner: a thread owns COLS float4 column groups for
// the whole launch and folds rows 0..N-1 into registers in order; PF rows are in flight
// (a register ring with static indices), so each lane keeps PF*COLS*16 B of loads outstanding.
// ------------------------------------------------------------------------------------------
template <class Op, int COLS, int PF, bool W>
__global__ __launch_bounds__(256) void k_ew_accum_vec(RowSrc src, int64_t n, int64_t d, Op op,
                                                      const float* __restrict__ levels, int s,
                                                      const float* __restrict__ w, float wt,
                                                      float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float4 smem_tab[];
    if (Op::TABLE) op.set_table_ok(load_table(levels, s, smem_tab));
    const int64_t groups = d / 4;
    const int64_t tile_groups = (int64_t)blockDim.x * COLS;
    for (int64_t t0 = (int64_t)blockIdx.x * tile_groups; t0 < groups; t0 += (int64_t)gridDim.x * tile_groups) {
        int64_t gi[COLS];
        bool ok[COLS];
        uint32_t cs[COLS][4];
#pragma unroll
        for (int c = 0; c < COLS; ++c) {
            gi[c] = t0 + threadIdx.x + c * 256;
            ok[c] = gi[c] < groups;
#pragma unroll
            for (int q = 0; q < 4; ++q) cs[c][q] = op.col(gi[c] * 4 + q);
        }
        float4 ring[PF][COLS];
#pragma unroll
        for (int p = 0; p < PF; ++p) {
            if (p < n) {
                const float4* r = reinterpret_cast<const float4*>(src.row(p));
#pragma unroll
                for (int c = 0; c < COLS; ++c) ring[p][c] = ok[c] ? ld_row4(r + gi[c]) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
        float4 acc[COLS];
        for (int64_t i0 = 0; i0 < n; i0 += PF) {
#pragma unroll
            for (int p = 0; p < PF; ++p) {
                const int64_t i = i0 + p;
                if (i < n) {
                    op.setup(i);
                    const float wi = W ? w[i] : 1.f;
                    float4 e[COLS];
                    if (op.row_fast())     // row-uniform: whole row inside the fast-division window
                        apply_cols<true, COLS>(op, ring[p], gi, cs, smem_tab, e);
                    else
                        apply_cols<false, COLS>(op, ring[p], gi, cs, smem_tab, e);
#pragma unroll
                    for (int c = 0; c < COLS; ++c) {
                        const float4 t = W ? make_float4(wi * e[c].x, wi * e[c].y, wi * e[c].z, wi * e[c].w) : e[c];
                        if (i == 0) acc[c] = t;
                        else {
                            acc[c].x = acc[c].x + t.x; acc[c].y = acc[c].y + t.y;
                            acc[c].z = acc[c].z + t.z; acc[c].w = acc[c].w + t.w;
                        }
                    }
                    if (i + PF < n) {
                        const float4* r = reinterpret_cast<const float4*>(src.row(i + PF));
#pragma unroll
                        for (int c = 0; c < COLS; ++c) ring[p][c] = ok[c] ? ld_row4(r + gi[c]) : make_float4(0.f, 0.f, 0.f, 0.f);
                    }
                }
            }
        }
#pragma unroll
        for (int c = 0; c < COLS; ++c)
            if (ok[c])
                reinterpret_cast<float4*>(out)[gi[c]] =
                    make_float4(acc[c].x / wt, acc[c].y / wt, acc[c].z / wt, acc[c].w / wt);
    }
}

template <class Op>
__global__ __launch_bounds__(256) void k_ew_accum_scalar(RowSrc src, int64_t n, int64_t j0, int64_t d, Op op,
                                                         const float* __restrict__ levels, int s,
                                                         const float* __restrict__ w, float wt,
                                                         float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float4 smem_tab[];
    if (Op::TABLE) op.set_table_ok(load_table(levels, s, smem_tab));
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t j = j0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += stride) {
        const uint32_t cs = op.col(j);
        float acc = 0.f;
        for (int64_t i = 0; i < n; ++i) {
            op.setup(i);
            const float t = (w ? w[i] : 1.f) * op.template apply<false>(src.row(i)[j], j, cs, smem_tab);
            acc = (i == 0) ? t : acc + t;
        }
        out[j] = acc / wt;
    }
}

// device-RNG row keys (natural codec; dithering gets them from k_norm_final)
__global__ void k_row_keys(int64_t n, uint64_t seed, int64_t client0, uint32_t* __restrict__ rk) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
        rk[r] = rowkey(client_key(seed, client0 + r));
}

static int grid_cap(int64_t work, int64_t per_block, int64_t cap) {
    int64_t b = (work + per_block - 1) / per_block;
    return (int)std::max<int64_t>(1, std::min<int64_t>(b, cap));
}

template <class Op>
static int launch_dense(const float* x, int64_t d, Op op, const float* levels, int s, float* out, hipStream_t st) {
    if (d == 0) return FLC_OK;
    const bool vec = (((uintptr_t)x | (uintptr_t)out) & 15u) == 0;
    const size_t lds = Op::TABLE ? (size_t)s * sizeof(float4) : 0;
    const int grid = grid_cap(vec ? (d + 3) / 4 : d, 256, 4096);
    if (vec) hipLaunchKernelGGL((k_ew_dense<Op, true>), dim3(grid), dim3(256), lds, st, x, d, op, levels, s, out);
    else hipLaunchKernelGGL((k_ew_dense<Op, false>), dim3(grid), dim3(256), lds, st, x, d, op, levels, s, out);
    FLC_CHECK_LAUNCH("k_ew_dense");
    return FLC_OK;
}

template <class Op>
static int launch_shift(const float* a, int64_t d, Op op, const float* levels, int s, const ShiftArgs& sh,
                        hipStream_t st) {
    if (d == 0) return FLC_OK;
    const uintptr_t al = (uintptr_t)a | (uintptr_t)sh.b | (uintptr_t)sh.base | (uintptr_t)sh.msg |
                         (uintptr_t)sh.hin | (uintptr_t)sh.hout;
    const bool vec = (al & 15u) == 0;
    const size_t lds = Op::TABLE ? (size_t)s * sizeof(float4) : 0;
    const int grid = grid_cap(vec ? (d + 3) / 4 : d, 256, 4096);
    ProfScope _ps("k_ew_shift", st);
    if (vec) hipLaunchKernelGGL((k_ew_shift<Op, true>), dim3(grid), dim3(256), lds, st, a, d, op, levels, s, sh);
    else hipLaunchKernelGGL((k_ew_shift<Op, false>), dim3(grid), dim3(256), lds, st, a, d, op, levels, s, sh);
    FLC_CHECK_LAUNCH("k_ew_shift");
    return FLC_OK;
}

// tile shape of the accumulate kernel: COLS float4 columns per thread, PF rows in flight;
// FLC_EW_TILE=<cols>x<pf> overrides (tuning runs only).
static int ew_tile_variant() {
    static int v = [] {
        const char* e = tuning_env("FLC_EW_TILE");
        if (!e) return 0;
        if (!strcmp(e, "2x2")) return 1;
        if (!strcmp(e, "2x4")) return 2;
        if (!strcmp(e, "1x8")) return 3;
        if (!strcmp(e, "1x4")) return 4;
        if (!strcmp(e, "4x2")) return 5;
        return 0;
    }();
    return v;
}

template <class Op, int COLS, int PF>
static int launch_accum_tile(RowSrc src, int64_t n, int64_t d, Op op, const float* levels, int s, const float* w,
                             float wt, float* out, size_t lds, hipStream_t st) {
    const int64_t groups = d / 4;
    const int grid = grid_cap(groups, 256 * COLS, 1 << 20);
    ProfScope _ps("k_ew_accum_vec", st);
    if (w) hipLaunchKernelGGL((k_ew_accum_vec<Op, COLS, PF, true>), dim3(grid), dim3(256), lds, st, src, n, d, op,
                              levels, s, w, wt, out);
    else hipLaunchKernelGGL((k_ew_accum_vec<Op, COLS, PF, false>), dim3(grid), dim3(256), lds, st, src, n, d, op,
                            levels, s, w, wt, out);
    return FLC_OK;
}

template <class Op>
static int launch_accum(RowSrc src, bool vec, int64_t n, int64_t d, Op op, const float* levels, int s,
                        const float* w, float wt, float* out, hipStream_t st) {
    if (d == 0) return FLC_OK;
    const size_t lds = Op::TABLE ? (size_t)s * sizeof(float4) : 0;
    int64_t j0 = 0;
    if (vec && ((uintptr_t)out & 15u) == 0) {
        if (d / 4 > 0) {
            switch (ew_tile_variant()) {
                case 2: launch_accum_tile<Op, 2, 4>(src, n, d, op, levels, s, w, wt, out, lds, st); break;
                case 3: launch_accum_tile<Op, 1, 8>(src, n, d, op, levels, s, w, wt, out, lds, st); break;
                case 4: launch_accum_tile<Op, 1, 4>(src, n, d, op, levels, s, w, wt, out, lds, st); break;
                case 5: launch_accum_tile<Op, 4, 2>(src, n, d, op, levels, s, w, wt, out, lds, st); break;
                default: launch_accum_tile<Op, 2, 2>(src, n, d, op, levels, s, w, wt, out, lds, st); break;  // measured best (C4)
            }
            FLC_CHECK_LAUNCH("k_ew_accum_vec");
        }
        j0 = (d / 4) * 4;
    }
    if (j0 < d) {
        const int grid = grid_cap(d - j0, 256, 4096);
        hipLaunchKernelGGL((k_ew_accum_scalar<Op>), dim3(grid), dim3(256), lds, st, src, n, j0, d, op, levels, s, w,
                           wt, out);
        FLC_CHECK_LAUNCH("k_ew_accum_scalar");
    }
    return FLC_OK;
}

// ------------------------------------------------------------------------------------------
// Entry points used by api.hip
// ------------------------------------------------------------------------------------------
struct EwWs {
    double* partial;
    uint32_t* tinyp;
    float* pn;
    float* rpn;
    uint32_t* fast;
    uint32_t* rk;
};
static EwWs carve_ew(void* base, int64_t n, int64_t d, size_t* bytes) {
    Carver c(base);
    const size_t np = (size_t)std::max<int64_t>(n, 1), parts = (size_t)std::max<int64_t>(norm_parts(n, d), 1);
    EwWs w;
    w.partial = c.take<double>(np * parts);
    w.tinyp = c.take<uint32_t>(np * parts);
    w.pn = c.take<float>(np);
    w.rpn = c.take<float>(np);
    w.fast = c.take<uint32_t>(np);
    w.rk = c.take<uint32_t>(np);
    if (bytes) *bytes = c.bytes();
    return w;
}

// the caller forced the sparse dithering path (flc_codec_params.flags hint)
static bool lone_sparse(const flc_codec_params* prm) { return (prm->flags & FLC_PATH_MASK) == FLC_PATH_SPARSE; }

size_t ew_workspace(const flc_codec_params* prm, int64_t n, int64_t d) {
    if (prm->codec == FLC_IDENT || prm->codec == FLC_LAZY) return 0;
    size_t b = 0;
    carve_ew(nullptr, n, d, &b);
    // fused dithering may take the sparse path (device draws; the pattern is not known here)
    if ((n > 1 || lone_sparse(prm)) && ds_eligible(prm, nullptr, n, d)) b = std::max(b, ds_workspace(prm, n, d));
    return b;
}

static int check_dither(const flc_codec_params* prm) {
    if (prm->s < 1 || !prm->d_levels) { set_error("dithering: need s >= 1 and levels"); return FLC_ERR_ARG; }
    if (prm->s > 8192) { set_error("dithering: s=%d above the LDS level table (8192)", prm->s); return FLC_ERR_UNSUPPORTED; }
    if (prm->norm != FLC_NORM_L1 && prm->norm != FLC_NORM_L2 && prm->norm != FLC_NORM_LINF) {
        set_error("dithering: p-norm %d not supported (1, 2, inf)", prm->norm);
        return FLC_ERR_UNSUPPORTED;
    }
    return FLC_OK;
}

#ifndef FLC_LONE_DITHER
#define FLC_LONE_DITHER 1
#endif
// compressVector of one row with standard dithering and its own norm: the partials, then
// k_lone_dither (the norm folded in every block, the encode with its loads batched)
static int launch_lone_dither(const flc_codec_params* prm, const UniformSrc& us, bool compat, const float* x, int64_t d,
                              EwWs& e, float* pnorm_out, float* out, int64_t client0, hipStream_t st) {
    const int64_t parts = (d + LONE_PLEN - 1) / LONE_PLEN;
    const RowSrc src{x, d, nullptr};
    const dim3 pg((unsigned)std::min<int64_t>(parts, 4096), 1);
    const int64_t n4 = d / 4;
    const int eg = (int)std::max<int64_t>(1, std::min<int64_t>((n4 + 256 * LONE_U - 1) / (256 * LONE_U), FLC_LONE_GRID));
    const size_t lds = (size_t)prm->s * sizeof(float4);
    auto go = [&](auto nk, auto cm) -> int {
        constexpr int NK = decltype(nk)::value;
        constexpr bool CM = decltype(cm)::value;
        { ProfScope _ps("k_norm_partials", st);
        hipLaunchKernelGGL((k_norm_partials<NK, true, false, (bool)FLC_LONE_KEEP>), pg, dim3(256), 0, st, src, nullptr, d, parts, LONE_PLEN,
                           e.partial, e.tinyp); }
        FLC_CHECK_LAUNCH("k_norm_partials");
        DitherOp<false, CM> op;
        op.us = us;
        op.rt = RowTabs{e.pn, e.rpn, e.fast, e.rk};
        op.s = prm->s;
        op.sf = (float)prm->s;
        op.tab_ok = false;
        { ProfScope _ps("k_lone_dither", st);
        hipLaunchKernelGGL((k_lone_dither<NK, CM>), dim3(eg), dim3(256), lds, st, x, d, op, prm->d_levels, prm->s, out,
                           e.partial, e.tinyp, parts, e.pn, e.rpn, e.fast, prm->seed, client0, e.rk, pnorm_out); }
        FLC_CHECK_LAUNCH("k_lone_dither");
        return FLC_OK;
    };
    using L2 = std::integral_constant<int, FLC_NORM_L2>;
    using L1 = std::integral_constant<int, FLC_NORM_L1>;
    using LI = std::integral_constant<int, FLC_NORM_LINF>;
    using T = std::true_type;
    using Fa = std::false_type;
    if (prm->norm == FLC_NORM_L2) return compat ? go(L2{}, T{}) : go(L2{}, Fa{});
    if (prm->norm == FLC_NORM_L1) return compat ? go(L1{}, T{}) : go(L1{}, Fa{});
    return compat ? go(LI{}, T{}) : go(LI{}, Fa{});
}

// One row encode (compressVector) or fused reduce over n rows (n >= 1).
int ew_run(const flc_codec_params* prm, const flc_pattern* pat, RowSrc src, bool vec, int64_t n, int64_t d,
           const float* pnorm_in, float* pnorm_out, bool dense, float* out, const float* w, float wt,
           void* ws, size_t ws_bytes, hipStream_t st, const ShiftArgs* sh, const CodeArgs* ca) {
    if ((sh || ca) && (!dense || n != 1)) { set_error("ew_run: the shift / code forms are one dense row"); return FLC_ERR_ARG; }
    const int codec = prm->codec;
    const bool compat = pat && pat->d_uniforms;
    const int64_t client0 = pat ? pat->client0 : 0;
    UniformSrc us{compat ? pat->d_uniforms : nullptr, (pat && pat->uniforms_ld) ? pat->uniforms_ld : d};
    auto go = [&](auto op, const float* levels, int s) -> int {
        if (sh) return launch_shift(src.base, d, op, levels, s, *sh, st);
        if (ca) return launch_code(src.base, d, op, levels, s, *ca, st);
        if (dense) return launch_dense(src.base, d, op, levels, s, out, st);
        return launch_accum(src, vec, n, d, op, levels, s, w, wt, out, st);
    };
    if (!dense && !pnorm_in && n > 1 && ds_eligible(prm, pat, n, d))
        return ds_run(prm, pat, src, n, d, w, wt, pnorm_out, out, ws, ws_bytes, st);
    // a lone compressVector row on the single-read sparse pass, when the caller forces it (the fold
    // of one row with weight 1 is the row's encode, -0 included: (1 * v) / 1 == v).  Not the
    // automatic choice: at D = 25 M the two-pass dense encode is 2.2 x faster (62 vs 218 us, device
    // draws; the one-row fold walks every tile of the row), profiles/r04/lone_ab.txt
    if (lone_sparse(prm) && dense && !sh && !ca && !pnorm_in && n == 1 && ds_eligible(prm, pat, 1, d))
        return ds_run(prm, pat, src, 1, d, nullptr, 1.f, pnorm_out, out, ws, ws_bytes, st);
    if (ws_bytes < ew_workspace(prm, n, d)) { set_error("codec workspace too small"); return FLC_ERR_WORKSPACE; }
    EwWs e = carve_ew(ws, n, d, nullptr);
    switch (codec) {
        case FLC_IDENT: {
            IdentOp op;
            return go(op, nullptr, 0);
        }
        case FLC_LAZY: {
            if (!pat || !pat->d_lazy_u) { set_error("lazy: pattern needs d_lazy_u"); return FLC_ERR_ARG; }
            LazyOp op;
            op.lazy_u = pat->d_lazy_u;
            op.P = prm->lazy_p;
            return go(op, nullptr, 0);
        }
        case FLC_NATURAL: {
            if (compat) { NaturalOp<true> op; op.us = us; op.rks = nullptr; return go(op, nullptr, 0); }
            hipLaunchKernelGGL(k_row_keys, dim3(grid_cap(n, 256, 64)), dim3(256), 0, st, n, prm->seed, client0, e.rk);
            FLC_CHECK_LAUNCH("k_row_keys");
            NaturalOp<false> op;
            op.us = us;
            op.rks = e.rk;
            return go(op, nullptr, 0);
        }
        case FLC_STD_DITHERING:
        case FLC_NAT_DITHERING: {
            int rc = check_dither(prm);
            if (rc) return rc;
            if (FLC_LONE_DITHER && codec == FLC_STD_DITHERING && dense && !sh && !ca && n == 1 && !pnorm_in &&
                ((((uintptr_t)src.base | (uintptr_t)out) & 15u) == 0) && (!compat || ((uintptr_t)us.u & 15u) == 0))
                return launch_lone_dither(prm, us, compat, src.base, d, e, pnorm_out, out, client0, st);
            RowTabs rt{pnorm_in, nullptr, nullptr, e.rk};
            if (!pnorm_in) {
                rc = launch_norms(src, vec, n, d, prm->norm, e.partial, e.tinyp, e.pn, e.rpn, e.fast, prm->seed,
                                  client0, e.rk, st, sh ? sh->b : nullptr);
                if (rc) return rc;
                rt = RowTabs{e.pn, e.rpn, e.fast, e.rk};
            } else if (!compat) {
                hipLaunchKernelGGL(k_row_keys, dim3(grid_cap(n, 256, 64)), dim3(256), 0, st, n, prm->seed, client0, e.rk);
                FLC_CHECK_LAUNCH("k_row_keys");
            }
            if (pnorm_out && pnorm_out != rt.pn)
                FLC_CHECK_HIP(hipMemcpyAsync(pnorm_out, rt.pn, (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, st));
            auto fill = [&](auto& op) {
                op.us = us; op.rt = rt; op.s = prm->s; op.sf = (float)prm->s; op.tab_ok = false;
            };
            if (codec == FLC_STD_DITHERING) {
                if (compat) { DitherOp<false, true> op; fill(op); return go(op, prm->d_levels, prm->s); }
                DitherOp<false, false> op;
                fill(op);
                return go(op, prm->d_levels, prm->s);
            }
            DitherOp<true, false> op;   // natural dithering output does not depend on the draws
            fill(op);
            return go(op, prm->d_levels, prm->s);
        }
        default:
            set_error("ew_run: codec %d is not elementwise", codec);
            return FLC_ERR_UNSUPPORTED;
    }
}

// ------------------------------------------------------------------------------------------
// Self-test of the fast division: for each divisor, every float numerator in [2^-80, 2^80] (the
// window div_rn / div_fast use) is divided both ways; mismatches are counted.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_selftest_div(const float* __restrict__ bs, int nb,
                                                      unsigned long long* __restrict__ bad) {
    const uint32_t lo = __float_as_uint(0x1p-80f), hi = __float_as_uint(0x1p80f);
    const uint64_t count = (uint64_t)(hi - lo) + 1;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (int k = 0; k < nb; ++k) {
        const FastDiv f = make_div(bs[k]);
        unsigned long long local = 0;
        for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < count; t += stride) {
            const float a = __uint_as_float(lo + (uint32_t)t);
            const float q = div_rn(a, f), r = a / f.b;
            local += (__float_as_uint(q) != __float_as_uint(r)) ? 1ull : 0ull;
        }
        local = wave_sum(local);
        if ((threadIdx.x & 63) == 0 && local) atomicAdd(&bad[k], local);
    }
}

int selftest_division(const float* d_b, int nb, unsigned long long* d_bad, hipStream_t st) {
    FLC_CHECK_HIP(hipMemsetAsync(d_bad, 0, (size_t)nb * sizeof(unsigned long long), st));
    hipLaunchKernelGGL(k_selftest_div, dim3(8192), dim3(256), 0, st, d_b, nb, d_bad);
    FLC_CHECK_LAUNCH("k_selftest_div");
    return FLC_OK;
}

// ------------------------------------------------------------------------------------------
// The fp32 2-norm in torch's CPU reduction order (compressors.py:272 `torch.norm(x, p=2)` on a
// CPU fp32 tensor; oracle/torch_norm.c restates it and tests/golden/rows.json pins it at D = 25 M):
// 8 lane accumulators, lane l taking x[8k + l]^2 in order as fused multiply-adds, the 8 lanes
// summed left to right, the D % 8 tail elements' squares added in order (fused), then the
// correctly rounded square root.  Each lane's sum is one chain of D / 8 dependent fmas, which
// no reassociation may shorten, so the kernel is built around that chain: one workgroup per row,
// wave 0's lanes 0..7 run the 8 chains out of LDS (transposed: a chain's 4 next steps are one
// ds_read_b128, 8 of them in flight) while waves 1..3 stream the next TN_CH elements into the
// other half of a double buffer with every float4 load of the chunk in flight at once (the
// previous form issued them a few at a time: 52.4 ms per call at D = 25 M, the chain waiting on
// the staging; a single-wave register ring, every step's 4-byte load issued 64 steps ahead, 33.4
// ms — a block of 64 steps does not cover one HBM latency).  Latency-bound by design: the parity
// mode of the drop-in, not a fast path.
// ------------------------------------------------------------------------------------------
constexpr int TN_CH = 16384;                // elements per staged chunk (2048 steps of each chain)
constexpr int TN_ST = TN_CH / 8 + 4;        // LDS stride of a lane's steps (+4: conflict-free staging)
constexpr int TN_LD = (TN_CH / 4 + 191) / 192;   // float4 loads per staging thread and chunk

__global__ __launch_bounds__(256) void k_norm_torch(const float* __restrict__ base, int64_t ld, int64_t d,
                                                    float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float tn_buf[];      // [2][8 * TN_ST]
    const int t = threadIdx.x;
    const int64_t row = blockIdx.x;
    const float* r = base + row * ld;
    const int64_t m = d - d % 8;                              // the lane accumulators' elements
    const int64_t nc = (m + TN_CH - 1) / TN_CH;
    // waves 1..3 stage chunk c: every float4 load first (range-checked: zeros past m, and
    // fmaf(0, 0, a) == a for the non-negative accumulators), then the transposed LDS writes
    auto stage = [&](int64_t c) {
        float* b = tn_buf + (c & 1) * 8 * TN_ST;
        const int64_t j0 = c * TN_CH;
        const int64_t left = m - j0;
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(r + j0), (short)0,
                                                          (int)(left >= TN_CH ? TN_CH * 4 : left * 4), 0x00020000);
        typedef unsigned int u4v __attribute__((ext_vector_type(4)));
        u4v q[TN_LD];
        const int p = t - 64;                                  // 0..191
#pragma unroll
        for (int u = 0; u < TN_LD; ++u) {
            const int f = p + u * 192;                         // float4 index in the chunk
            q[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(f < TN_CH / 4 ? f : 0) * 16u, 0, 2);
        }
#pragma unroll
        for (int u = 0; u < TN_LD; ++u) {
            const int f = p + u * 192;
            if (f < TN_CH / 4) {
                const int k = f >> 1, l0 = (f & 1) * 4;        // elements 4f .. 4f+3 = steps k of lanes l0 ..
#pragma unroll
                for (int e = 0; e < 4; ++e) b[(l0 + e) * TN_ST + k] = __uint_as_float(q[u][e]);
            }
        }
    };
    float acc = 0.f;
    if (t >= 64 && nc > 0) stage(0);
    __syncthreads();
    for (int64_t c = 0; c < nc; ++c) {
        if (t >= 64) {
            if (c + 1 < nc) stage(c + 1);
        } else if (t < 8) {
            const float4* b4 = reinterpret_cast<const float4*>(tn_buf + (c & 1) * 8 * TN_ST + t * TN_ST);
            constexpr int R = 8;                               // ds_read_b128 in flight
            float4 cur[R];
#pragma unroll
            for (int u = 0; u < R; ++u) cur[u] = b4[u];
            for (int s = 0; s < TN_CH / 32; s += R) {
                float4 nxt[R];
#pragma unroll
                for (int u = 0; u < R; ++u) nxt[u] = b4[(s + R + u) % (TN_CH / 32)];   // (the wrap re-reads: harmless)
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
        __syncthreads();
    }
    if (t < 64) {
        float tot = __shfl(acc, 0, 64);
        for (int l = 1; l < 8; ++l) tot = tot + __shfl(acc, l, 64);   // buffer[0] + buffer[1] + ...
        if (t == 0) {
            for (int64_t k = m; k < d; ++k) tot = fmaf(r[k], r[k], tot);
            out[row] = (float)sqrt((double)tot);               // RN(sqrt): exact via double
        }
    }
}

int norm_torch_run(const float* x, int64_t ld, int64_t n, int64_t d, float* out, hipStream_t st) {
    if (n <= 0) return FLC_OK;
    ProfScope _ps("k_norm_torch", st);
    const size_t lds = 2 * 8 * TN_ST * sizeof(float);          // 128 KB: the double buffer
    static const bool ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_norm_torch),
                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess;
    if (!ok) { set_error("k_norm_torch: %zu bytes of dynamic LDS refused", lds); return FLC_ERR_HIP; }
    hipLaunchKernelGGL(k_norm_torch, dim3((unsigned)n), dim3(256), lds, st, x, ld, d, out);
    FLC_CHECK_LAUNCH("k_norm_torch");
    return FLC_OK;
}

}  // namespace flc
