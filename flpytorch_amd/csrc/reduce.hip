// N-way reduction — the serverGradient core (fl_pytorch/utils/algorithms.py:1753-1768).
//
//   REL_X : out = (w0*(x - r0) (+) w1*(x - r1) (+) ...) / w_total
//   PLAIN : out = (w0*r0 (+) w1*r1 (+) ...) / w_total
//
// Per element the rows are folded strictly in row order with one fp32 rounding per operation
// (the library is built with -ffp-contract=off), which is exactly the reference's sequential
// torch loop: bit-identical results.  HBM-bound: 4*N*D bytes read + 4*D written.
//
// Layout/launch: each thread owns one float4 column group and walks all N rows; rows are
// fetched UNROLL at a time so UNROLL*16 B per lane are in flight; a wave reads 1 KB contiguous
// per row per instruction.  Grid-stride over column groups, ~2 K workgroups (>> 256 CUs).
#include "common.hpp"

namespace flc {

template <int MODE>
__device__ inline float4 term(float4 r, float4 x, float w) {
    float4 g = r;
    if (MODE == FLC_REDUCE_REL_X) { g.x = x.x - r.x; g.y = x.y - r.y; g.z = x.z - r.z; g.w = x.w - r.w; }
    return make_float4(w * g.x, w * g.y, w * g.z, w * g.w);
}

template <int MODE, int UNROLL>
__global__ __launch_bounds__(256) void k_reduce_vec(RowSrc src, int64_t n, int64_t groups,
                                                    const float* __restrict__ x,
                                                    const float* __restrict__ w, float wt,
                                                    float* __restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < groups; g += stride) {
        float4 xv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (MODE == FLC_REDUCE_REL_X) xv = reinterpret_cast<const float4*>(x)[g];
        float4 acc;
        {
            float4 r = ld_row4(reinterpret_cast<const float4*>(src.row(0)) + g);
            acc = term<MODE>(r, xv, w ? w[0] : 1.f);
        }
        int64_t i = 1;
        for (; i + UNROLL <= n; i += UNROLL) {
            float4 r[UNROLL];
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) r[u] = ld_row4(reinterpret_cast<const float4*>(src.row(i + u)) + g);
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                float4 t = term<MODE>(r[u], xv, w ? w[i + u] : 1.f);
                acc.x = acc.x + t.x; acc.y = acc.y + t.y; acc.z = acc.z + t.z; acc.w = acc.w + t.w;
            }
        }
        for (; i < n; ++i) {
            float4 t = term<MODE>(ld_row4(reinterpret_cast<const float4*>(src.row(i)) + g), xv, w ? w[i] : 1.f);
            acc.x = acc.x + t.x; acc.y = acc.y + t.y; acc.z = acc.z + t.z; acc.w = acc.w + t.w;
        }
        reinterpret_cast<float4*>(out)[g] = make_float4(acc.x / wt, acc.y / wt, acc.z / wt, acc.w / wt);
    }
}

// Scalar path: any alignment / any d (also the tail of the vector path).
template <int MODE>
__global__ __launch_bounds__(256) void k_reduce_scalar(RowSrc src, int64_t n, int64_t j0, int64_t d,
                                                       const float* __restrict__ x,
                                                       const float* __restrict__ w, float wt,
                                                       float* __restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t j = j0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += stride) {
        const float xv = (MODE == FLC_REDUCE_REL_X) ? x[j] : 0.f;
        float acc = 0.f;
        for (int64_t i = 0; i < n; ++i) {
            float r = src.row(i)[j];
            float g = (MODE == FLC_REDUCE_REL_X) ? xv - r : r;
            float t = (w ? w[i] : 1.f) * g;
            acc = (i == 0) ? t : acc + t;
        }
        out[j] = acc / wt;
    }
}

static int grid_for(int64_t work, int64_t cap = 2048) {
    int64_t b = (work + 255) / 256;
    if (b < 1) b = 1;
    if (b > cap) b = cap;
    return (int)b;
}

template <int MODE>
static int launch_reduce(RowSrc src, bool vec_ok, int64_t n, int64_t d, const float* x, const float* w,
                         float wt, float* out, hipStream_t st) {
    int64_t j0 = 0;
    if (vec_ok) {
        int64_t groups = d / 4;
        if (groups > 0) {
{ ProfScope _ps("k_reduce_vec", st);
            hipLaunchKernelGGL((k_reduce_vec<MODE, 8>), dim3(grid_for(groups)), dim3(256), 0, st, src, n,
                               groups, x, w, wt, out); }
            FLC_CHECK_LAUNCH("k_reduce_vec");
        }
        j0 = groups * 4;
    }
    if (j0 < d) {
        hipLaunchKernelGGL((k_reduce_scalar<MODE>), dim3(grid_for(d - j0)), dim3(256), 0, st, src, n, j0, d, x,
                           w, wt, out);
        FLC_CHECK_LAUNCH("k_reduce_scalar");
    }
    return FLC_OK;
}

static bool al16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

int reduce_impl(RowSrc src, bool rows_vec_ok, int64_t n, int64_t d, const float* x, const float* w,
                float wt, int mode, float* out, hipStream_t st) {
    if (n < 0 || d < 0 || !out) { set_error("flc_reduce: bad n/d/out"); return FLC_ERR_ARG; }
    if (mode != FLC_REDUCE_PLAIN && mode != FLC_REDUCE_REL_X) { set_error("flc_reduce: bad mode %d", mode); return FLC_ERR_ARG; }
    if (mode == FLC_REDUCE_REL_X && !x) { set_error("flc_reduce: REL_X needs x"); return FLC_ERR_ARG; }
    if (d == 0) return FLC_OK;
    if (n == 0) {   // algorithms.py:2117-2118: no clients -> zeros_like(x)
        FLC_CHECK_HIP(hipMemsetAsync(out, 0, (size_t)d * sizeof(float), st));
        return FLC_OK;
    }
    bool vec = rows_vec_ok && al16(out) && (mode == FLC_REDUCE_PLAIN || al16(x));
    if (mode == FLC_REDUCE_REL_X) return launch_reduce<FLC_REDUCE_REL_X>(src, vec, n, d, x, w, wt, out, st);
    return launch_reduce<FLC_REDUCE_PLAIN>(src, vec, n, d, x, w, wt, out, st);
}

}  // namespace flc

using namespace flc;

extern "C" int flc_reduce_rows(const float* const* d_row_ptrs, int64_t n, int64_t d, const float* d_x,
                               const float* d_w, float w_total, int mode, float* d_out, void* stream) {
    if (n > 0 && !d_row_ptrs) { set_error("flc_reduce_rows: null row pointer array"); return FLC_ERR_ARG; }
    RowSrc src{nullptr, 0, d_row_ptrs};
    // Row pointers are device data: the caller asserts 16-byte alignment by passing rows that are
    // (torch allocations are); the Python layer checks each data_ptr before choosing this entry.
    return reduce_impl(src, true, n, d, d_x, d_w, w_total, mode, d_out, (hipStream_t)stream);
}

extern "C" int flc_reduce_matrix(const float* d_rows, int64_t ld, int64_t n, int64_t d, const float* d_x,
                                 const float* d_w, float w_total, int mode, float* d_out, void* stream) {
    if (n > 0 && (!d_rows || ld < d)) { set_error("flc_reduce_matrix: null rows or ld < d"); return FLC_ERR_ARG; }
    RowSrc src{d_rows, ld, nullptr};
    bool vec = al16(d_rows) && (ld % 4 == 0);
    return reduce_impl(src, vec, n, d, d_x, d_w, w_total, mode, d_out, (hipStream_t)stream);
}
