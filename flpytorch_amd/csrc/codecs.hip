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
#include "common.hpp"

namespace flc {

// ------------------------------------------------------------------------------------------
// p-norms: partial[row][part] (float64, fixed slots) then one wave per row folds them in a
// fixed order -> deterministic, exactly rounded fp32 norm.
// ------------------------------------------------------------------------------------------
constexpr int NORM_PART = 65536;   // elements per partial (256 threads x 64 elements)

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

template <int NORM, bool VEC>
__global__ __launch_bounds__(256) void k_norm_partials(RowSrc src, int64_t d, int64_t parts,
                                                       double* __restrict__ partial) {
    const int64_t row = blockIdx.y;
    const float* r = src.row(row);
    __shared__ double red[4];
    for (int64_t part = blockIdx.x; part < parts; part += gridDim.x) {
        const int64_t j0 = part * NORM_PART;
        const int64_t j1 = min(d, j0 + (int64_t)NORM_PART);
        double a = 0.0;
        if (VEC) {
            const int64_t g0 = j0 / 4, g1 = j1 / 4;   // j0 % 4 == 0 (NORM_PART % 4 == 0)
            for (int64_t g = g0 + threadIdx.x; g < g1; g += 256) {
                float4 v = reinterpret_cast<const float4*>(r)[g];
                a = nacc<NORM>(a, v.x); a = nacc<NORM>(a, v.y); a = nacc<NORM>(a, v.z); a = nacc<NORM>(a, v.w);
            }
            for (int64_t j = g1 * 4 + threadIdx.x; j < j1; j += 256) a = nacc<NORM>(a, r[j]);
        } else {
            for (int64_t j = j0 + threadIdx.x; j < j1; j += 256) a = nacc<NORM>(a, r[j]);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) a = ncomb<NORM>(a, __shfl_xor(a, o, WAVE));
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
        __syncthreads();
        if (threadIdx.x == 0)
            partial[row * parts + part] = ncomb<NORM>(ncomb<NORM>(red[0], red[1]), ncomb<NORM>(red[2], red[3]));
        __syncthreads();
    }
}

template <int NORM>
__global__ __launch_bounds__(64) void k_norm_final(const double* __restrict__ partial, int64_t parts,
                                                   int64_t n, float* __restrict__ pn) {
    const int64_t row = blockIdx.x;
    if (row >= n) return;
    double a = 0.0;
    for (int64_t p = threadIdx.x; p < parts; p += 64) a = ncomb<NORM>(a, partial[row * parts + p]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) a = ncomb<NORM>(a, __shfl_xor(a, o, WAVE));
    if (threadIdx.x == 0) pn[row] = (NORM == FLC_NORM_L2) ? (float)sqrt(a) : (float)a;
}

int64_t norm_parts(int64_t d) { return (d + NORM_PART - 1) / NORM_PART; }

int launch_norms(RowSrc src, bool vec, int64_t n, int64_t d, int norm, double* partial, float* pn,
                 hipStream_t st) {
    const int64_t parts = norm_parts(d);
    if (n == 0) return FLC_OK;
    if (parts == 0) {  // d == 0: norm of an empty vector
        FLC_CHECK_HIP(hipMemsetAsync(pn, 0, (size_t)n * sizeof(float), st));
        return FLC_OK;
    }
    dim3 grid((unsigned)std::min<int64_t>(parts, 64), (unsigned)n);
#define FLC_NORM_CASE(NK)                                                                           \
    { ProfScope _ps("k_norm_partials", st);                                                         \
    if (vec) hipLaunchKernelGGL((k_norm_partials<NK, true>), grid, dim3(256), 0, st, src, d, parts, partial); \
    else hipLaunchKernelGGL((k_norm_partials<NK, false>), grid, dim3(256), 0, st, src, d, parts, partial); }  \
    FLC_CHECK_LAUNCH("k_norm_partials");                                                            \
    hipLaunchKernelGGL((k_norm_final<NK>), dim3((unsigned)n), dim3(64), 0, st, partial, parts, n, pn);  \
    FLC_CHECK_LAUNCH("k_norm_final");
    if (norm == FLC_NORM_L2) { FLC_NORM_CASE(FLC_NORM_L2) }
    else if (norm == FLC_NORM_L1) { FLC_NORM_CASE(FLC_NORM_L1) }
    else { FLC_NORM_CASE(FLC_NORM_LINF) }
#undef FLC_NORM_CASE
    return FLC_OK;
}

// ------------------------------------------------------------------------------------------
// Per-element codec functors.  setup(row) reads the row-uniform state; apply(x, row, j) -> C(x).
// ------------------------------------------------------------------------------------------
struct UniformSrc {
    const double* u;      // compat: [n][uld] float64 numpy draws; nullptr -> device RNG
    int64_t uld;
    uint64_t seed;
    int64_t client0;
};

struct IdentOp {
    __device__ inline void setup(int64_t) {}
    __device__ inline float apply(float x, int64_t) const { return x; }
};

struct LazyOp {                       // compressors.py:231-238: x / P if testp < P else 0
    const double* lazy_u;             // [n] float64 draws (numpy random())
    float P;
    bool keep;
    __device__ inline void setup(int64_t row) { keep = lazy_u[row] < (double)P; }
    __device__ inline float apply(float x, int64_t) const { return keep ? x / P : 0.f; }
};

struct NaturalOp {                    // compressors.py:247-268
    UniformSrc us;
    const double* urow;
    uint64_t ckey;
    __device__ inline void setup(int64_t row) {
        urow = us.u ? us.u + row * us.uld : nullptr;
        ckey = client_key(us.seed, us.client0 + row);
    }
    __device__ inline float apply(float x, int64_t j) const {
        const float ax = fabsf(x);
        const float alpha = (float)log2((double)ax);          // correctly rounded fp32 log2
        const float lo = floorf(alpha), hi = ceilf(alpha);
        const float plo = exp2f(lo), phi = exp2f(hi);         // exact for integral exponents
        const float pt = (phi - ax) / plo;
        const double u = urow ? urow[j] : uniform53(ckey, j);
        const bool down = u < (double)pt;
        float out = tsign(x) * (down ? plo : phi);
        return (x == 0.f) ? 0.f : out;
    }
};

// Standard / natural dithering (compressors.py:270-329).  levels in LDS as {l[s], l[s+1], l[s]-l[s+1]}.
template <bool NATBUG>
struct DitherOp {
    UniformSrc us;
    const float* pnorms;   // [n] fp32 norms
    const float4* tab;     // LDS table, s entries
    int s;
    float pn;
    const double* urow;
    uint64_t ckey;
    __device__ inline void setup(int64_t row) {
        pn = pnorms[row];
        urow = us.u ? us.u + row * us.uld : nullptr;
        ckey = client_key(us.seed, us.client0 + row);
    }
    __device__ inline float apply(float x, int64_t j) const {
        const float y = fabsf(x) / pn;
        if (NATBUG) return (y * tsign(x)) * pn;              // compressors.py:326
        float lev = 0.f;                                      // no interval matched -> 0
        if (y >= 0.f && y <= 1.f) {                           // levels span exactly [0, 1]
            int g = (int)(y * (float)s);
            g = g < 0 ? 0 : (g > s - 1 ? s - 1 : g);
            float4 t = tab[g];
            while (g > 0 && y < t.x) t = tab[--g];
            while (g < s - 1 && y > t.y) t = tab[++g];
            if (y >= t.x && y <= t.y) {
                const float p = (y - t.y) / t.z;
                const double u = urow ? urow[j] : uniform53(ckey, j);
                lev = (u < (double)p) ? t.x : t.y;
            }
        }
        if (x == 0.f) lev = 0.f;
        return (lev * tsign(x)) * pn;
    }
};

// Natural-dithering levels are not uniform: the (int)(y*s) guess is then refined by the loops
// above; with levels 2^-k the walk is bounded by s.  A binary search would be shorter for large
// s; s <= 32 in practice (nat.dithering:10 in the reference's GUI list).

template <class Op>
__device__ inline float4 apply4(const Op& op, float4 v, int64_t j) {
    return make_float4(op.apply(v.x, j), op.apply(v.y, j + 1), op.apply(v.z, j + 2), op.apply(v.w, j + 3));
}

// ------------------------------------------------------------------------------------------
// Dense encode of one row (compressVector).
// ------------------------------------------------------------------------------------------
template <class Op, bool VEC>
__global__ __launch_bounds__(256) void k_ew_dense(const float* __restrict__ x, int64_t d, Op op,
                                                  const float* __restrict__ levels, float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float4 smem_tab[];
    if (levels) {   // dithering table
        int s = op.s_for_table();
        for (int i = threadIdx.x; i < s; i += blockDim.x)
            smem_tab[i] = make_float4(levels[i], levels[i + 1], levels[i] - levels[i + 1], 0.f);
        __syncthreads();
        op.bind_table(smem_tab);
    }
    op.setup(0);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    if (VEC) {
        const int64_t groups = d / 4;
        for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < groups; g += stride)
            reinterpret_cast<float4*>(out)[g] = apply4(op, reinterpret_cast<const float4*>(x)[g], g * 4);
        for (int64_t j = groups * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += stride)
            out[j] = op.apply(x[j], j);
    } else {
        for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += stride)
            out[j] = op.apply(x[j], j);
    }
}

// ------------------------------------------------------------------------------------------
// Fused encode + reduce over N rows (tile owner, rows folded in order).
// ------------------------------------------------------------------------------------------
template <class Op, int COLS>
__global__ __launch_bounds__(256) void k_ew_accum_vec(RowSrc src, int64_t n, int64_t d, Op op,
                                                      const float* __restrict__ levels,
                                                      const float* __restrict__ w, float wt,
                                                      float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float4 smem_tab[];
    if (levels) {
        int s = op.s_for_table();
        for (int i = threadIdx.x; i < s; i += blockDim.x)
            smem_tab[i] = make_float4(levels[i], levels[i + 1], levels[i] - levels[i + 1], 0.f);
        __syncthreads();
        op.bind_table(smem_tab);
    }
    const int64_t groups = d / 4;
    const int64_t tile_groups = (int64_t)blockDim.x * COLS;
    for (int64_t t0 = (int64_t)blockIdx.x * tile_groups; t0 < groups; t0 += (int64_t)gridDim.x * tile_groups) {
        // thread's column groups: t0 + threadIdx.x + c*256 (coalesced per c)
        float4 acc[COLS];
        float4 cur[COLS];
        bool ok[COLS];
#pragma unroll
        for (int c = 0; c < COLS; ++c) ok[c] = (t0 + threadIdx.x + c * 256) < groups;
        {
            const float4* r0 = reinterpret_cast<const float4*>(src.row(0));
#pragma unroll
            for (int c = 0; c < COLS; ++c) cur[c] = ok[c] ? r0[t0 + threadIdx.x + c * 256] : make_float4(0, 0, 0, 0);
        }
        for (int64_t i = 0; i < n; ++i) {
            float4 nxt[COLS];
            if (i + 1 < n) {
                const float4* rn = reinterpret_cast<const float4*>(src.row(i + 1));
#pragma unroll
                for (int c = 0; c < COLS; ++c) nxt[c] = ok[c] ? rn[t0 + threadIdx.x + c * 256] : make_float4(0, 0, 0, 0);
            }
            op.setup(i);
            const float wi = w ? w[i] : 1.f;
#pragma unroll
            for (int c = 0; c < COLS; ++c) {
                const int64_t j = (t0 + threadIdx.x + c * 256) * 4;
                float4 e = apply4(op, cur[c], j);
                float4 t = make_float4(wi * e.x, wi * e.y, wi * e.z, wi * e.w);
                if (i == 0) acc[c] = t;
                else { acc[c].x = acc[c].x + t.x; acc[c].y = acc[c].y + t.y; acc[c].z = acc[c].z + t.z; acc[c].w = acc[c].w + t.w; }
            }
            if (i + 1 < n) {
#pragma unroll
                for (int c = 0; c < COLS; ++c) cur[c] = nxt[c];
            }
        }
#pragma unroll
        for (int c = 0; c < COLS; ++c)
            if (ok[c])
                reinterpret_cast<float4*>(out)[t0 + threadIdx.x + c * 256] =
                    make_float4(acc[c].x / wt, acc[c].y / wt, acc[c].z / wt, acc[c].w / wt);
    }
}

template <class Op>
__global__ __launch_bounds__(256) void k_ew_accum_scalar(RowSrc src, int64_t n, int64_t j0, int64_t d, Op op,
                                                         const float* __restrict__ levels,
                                                         const float* __restrict__ w, float wt,
                                                         float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float4 smem_tab[];
    if (levels) {
        int s = op.s_for_table();
        for (int i = threadIdx.x; i < s; i += blockDim.x)
            smem_tab[i] = make_float4(levels[i], levels[i + 1], levels[i] - levels[i + 1], 0.f);
        __syncthreads();
        op.bind_table(smem_tab);
    }
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t j = j0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += stride) {
        float acc = 0.f;
        for (int64_t i = 0; i < n; ++i) {
            op.setup(i);
            float t = (w ? w[i] : 1.f) * op.apply(src.row(i)[j], j);
            acc = (i == 0) ? t : acc + t;
        }
        out[j] = acc / wt;
    }
}

// Table plumbing for the functors (only dithering uses it).
template <class Base>
struct WithTable : Base {
    int s_tab = 0;
    __device__ inline int s_for_table() const { return s_tab; }
    __device__ inline void bind_table(const float4*) {}
};
template <bool NB>
struct DitherT : DitherOp<NB> {
    __device__ inline int s_for_table() const { return this->s; }
    __device__ inline void bind_table(const float4* t) { this->tab = t; }
};

static int grid_cap(int64_t work, int64_t per_block, int64_t cap) {
    int64_t b = (work + per_block - 1) / per_block;
    return (int)std::max<int64_t>(1, std::min<int64_t>(b, cap));
}

template <class Op>
static int launch_dense(const float* x, int64_t d, Op op, const float* levels, int s, float* out, hipStream_t st) {
    if (d == 0) return FLC_OK;
    const bool vec = (((uintptr_t)x | (uintptr_t)out) & 15u) == 0;
    size_t lds = levels ? (size_t)s * sizeof(float4) : 0;
    int grid = grid_cap(vec ? (d + 3) / 4 : d, 256, 4096);
    if (vec) hipLaunchKernelGGL((k_ew_dense<Op, true>), dim3(grid), dim3(256), lds, st, x, d, op, levels, out);
    else hipLaunchKernelGGL((k_ew_dense<Op, false>), dim3(grid), dim3(256), lds, st, x, d, op, levels, out);
    FLC_CHECK_LAUNCH("k_ew_dense");
    return FLC_OK;
}

template <class Op>
static int launch_accum(RowSrc src, bool vec, int64_t n, int64_t d, Op op, const float* levels, int s,
                        const float* w, float wt, float* out, hipStream_t st) {
    if (d == 0) return FLC_OK;
    size_t lds = levels ? (size_t)s * sizeof(float4) : 0;
    int64_t j0 = 0;
    if (vec && ((uintptr_t)out & 15u) == 0) {
        constexpr int COLS = 4;
        const int64_t groups = d / 4;
        if (groups > 0) {
            int grid = grid_cap(groups, 256 * COLS, 1 << 20);
{ ProfScope _ps("k_ew_accum_vec", st);
            hipLaunchKernelGGL((k_ew_accum_vec<Op, COLS>), dim3(grid), dim3(256), lds, st, src, n, d, op, levels, w,
                               wt, out); }
            FLC_CHECK_LAUNCH("k_ew_accum_vec");
        }
        j0 = groups * 4;
    }
    if (j0 < d) {
        int grid = grid_cap(d - j0, 256, 4096);
        hipLaunchKernelGGL((k_ew_accum_scalar<Op>), dim3(grid), dim3(256), lds, st, src, n, j0, d, op, levels, w, wt,
                           out);
        FLC_CHECK_LAUNCH("k_ew_accum_scalar");
    }
    return FLC_OK;
}

// ------------------------------------------------------------------------------------------
// Entry points used by api.hip
// ------------------------------------------------------------------------------------------
size_t ew_workspace(const flc_codec_params* prm, int64_t n, int64_t d) {
    Carver c(nullptr);
    if (prm->codec == FLC_STD_DITHERING || prm->codec == FLC_NAT_DITHERING) {
        c.take<double>((size_t)std::max<int64_t>(n, 1) * std::max<int64_t>(norm_parts(d), 1));
        c.take<float>((size_t)std::max<int64_t>(n, 1));
    }
    return c.bytes();
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

// One row encode (compressVector) or fused reduce over n rows (n >= 1).
int ew_run(const flc_codec_params* prm, const flc_pattern* pat, RowSrc src, bool vec, int64_t n, int64_t d,
           const float* pnorm_in, float* pnorm_out, bool dense, float* out, const float* w, float wt,
           void* ws, size_t ws_bytes, hipStream_t st) {
    const int codec = prm->codec;
    UniformSrc us{pat ? pat->d_uniforms : nullptr, (pat && pat->uniforms_ld) ? pat->uniforms_ld : d,
                  prm->seed, pat ? pat->client0 : 0};
    auto go = [&](auto op, const float* levels, int s) -> int {
        if (dense) return launch_dense(src.base, d, op, levels, s, out, st);
        return launch_accum(src, vec, n, d, op, levels, s, w, wt, out, st);
    };
    switch (codec) {
        case FLC_IDENT: {
            WithTable<IdentOp> op;
            return go(op, nullptr, 0);
        }
        case FLC_LAZY: {
            if (!pat || !pat->d_lazy_u) { set_error("lazy: pattern needs d_lazy_u"); return FLC_ERR_ARG; }
            WithTable<LazyOp> op;
            op.lazy_u = pat->d_lazy_u;
            op.P = prm->lazy_p;
            return go(op, nullptr, 0);
        }
        case FLC_NATURAL: {
            WithTable<NaturalOp> op;
            op.us = us;
            return go(op, nullptr, 0);
        }
        case FLC_STD_DITHERING:
        case FLC_NAT_DITHERING: {
            int rc = check_dither(prm);
            if (rc) return rc;
            if (ws_bytes < ew_workspace(prm, n, d)) { set_error("dithering: workspace too small"); return FLC_ERR_WORKSPACE; }
            Carver c(ws);
            double* partial = c.take<double>((size_t)std::max<int64_t>(n, 1) * std::max<int64_t>(norm_parts(d), 1));
            float* pn = c.take<float>((size_t)std::max<int64_t>(n, 1));
            const float* pn_use = pnorm_in;
            if (!pn_use) {
                rc = launch_norms(src, vec, n, d, prm->norm, partial, pn, st);
                if (rc) return rc;
                pn_use = pn;
            }
            if (pnorm_out && pnorm_out != pn_use)
                FLC_CHECK_HIP(hipMemcpyAsync(pnorm_out, pn_use, (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, st));
            if (codec == FLC_STD_DITHERING) {
                DitherT<false> op;
                op.us = us; op.pnorms = pn_use; op.s = prm->s; op.tab = nullptr;
                return go(op, prm->d_levels, prm->s);
            }
            DitherT<true> op;
            op.us = us; op.pnorms = pn_use; op.s = prm->s; op.tab = nullptr;
            return go(op, prm->d_levels, prm->s);
        }
        default:
            set_error("ew_run: codec %d is not elementwise", codec);
            return FLC_ERR_UNSUPPORTED;
    }
}

}  // namespace flc
