// Rank-K codec (fl_pytorch/utils/compressors.py:336-364): x viewed as the row-major A x B matrix X
// (makeRankKCompressor, 151-172: A = the smallest divisor of D that is >= int(D ** 0.5), B = D / A),
// truncated SVD with K' = min(K, min(A, B)) triplets:  out = (U_K diag(S_K)) V^T_K, flattened.
//
// The only dense-contraction codec of the reference: a thin SVD (rocSOLVER gesvd, batched over the
// clients) and one GEMM per row (rocBLAS).  Layout: the row-major X is the column-major B x A matrix
// M = X^T, so no transposes are materialised: M = U' S V'^T (U' is B x r, V'^T is r x A) gives
// X = V' S U'^T, and the reference's  (Uk diag(Sk)) Vtk = (V'_K diag S_K) U'^T_K  is, column-major,
//     C = M_K = U'_K (diag(S_K) V'^T_K)   (B x A, ldc = B),
// whose memory is exactly the row-major A x B result.  The rows of V'^T are scaled by S first: the
// same fp32 products the reference forms in Uk @ diag(Sk).  SVD factors are unique up to signs that
// cancel in the product; parity is stated to a tolerance (tests/test_gpu_rank_k.py).  A row whose
// SVD does not converge (rocSOLVER info > 0) keeps the partial factorisation, like LAPACK; the
// reference's retry on the CPU (339-347) has no counterpart.
//
// Factor blocks: every path reconstructs from one layout, the rank-K dyadic expansion the reference
// counts as K (A + B) sent values (compressors.py:362): per row U'_K (B x K, column-major, ld B),
// padded to 16 B, then (S V'^T)_K (K x A, column-major, ld K).  The encode writes the blocks to
// the workspace, flc_pack writes them as the payload body (wire.hip), and the one GEMM shape
// C = U'_K (S V'^T)_K reconstructs from either — so the decode of a payload is the encode, bit for
// bit.
//
// Memory: every buffer, including rocBLAS / rocSOLVER's own device memory (sized through the
// handle's size-query mode), comes from the caller's workspace.
#include <math.h>

#include <map>
#include <mutex>

#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include "common.hpp"

namespace flc {

struct RkShape {
    int64_t A, B, r, K;
};

static RkShape rk_shape(int64_t d, int64_t k) {
    RkShape s;
    int64_t a = (int64_t)sqrt((double)d);   // int(D ** 0.5): the float64 square root, truncated
    if (a < 1) a = 1;
    while (d % a != 0) ++a;
    s.A = a;
    s.B = d / a;
    s.r = std::min(s.A, s.B);
    s.K = std::max<int64_t>(0, std::min(k, s.r));
    return s;
}

namespace {
std::mutex g_rk_mu;
std::map<int, rocblas_handle> g_rk_handle;

rocblas_handle rk_handle() {    // caller holds g_rk_mu
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    rocblas_handle& h = g_rk_handle[dev];
    if (!h && rocblas_create_handle(&h) != rocblas_status_success) h = nullptr;
    return h;
}
}  // namespace

__host__ __device__ inline int64_t rk_uoff(const RkShape& sh) { return (sh.B * sh.K + 3) & ~int64_t(3); }
__host__ __device__ inline int64_t rk_block(const RkShape& sh) { return rk_uoff(sh) + ((sh.K * sh.A + 3) & ~int64_t(3)); }

struct RkWs {
    float* blk;     // [n][rk_block] factor blocks
    float* m;       // [n][D]   copy of the rows (gesvd overwrites its input)
    float* s;       // [n][r]
    float* u;       // [n][B * r]
    float* vt;      // [n][r * A]
    float* e;       // [n][r]
    rocblas_int* info;
    float* c;       // [n][D]   reconstructed rows (fused reduce only)
    void* lib;      // rocBLAS / rocSOLVER device memory
    size_t lib_bytes;
};

static RkWs carve_rk(void* base, const RkShape& sh, int64_t n, int64_t d, bool reduce, size_t lib_bytes,
                     size_t* bytes) {
    Carver cv(base);
    const size_t nn = (size_t)std::max<int64_t>(n, 1);
    RkWs w;
    w.blk = cv.take<float>(nn * std::max<int64_t>(rk_block(sh), 1));
    w.m = cv.take<float>(nn * d);
    w.s = cv.take<float>(nn * sh.r);
    w.u = cv.take<float>(nn * sh.B * sh.r);
    w.vt = cv.take<float>(nn * sh.r * sh.A);
    w.e = cv.take<float>(nn * sh.r);
    w.info = cv.take<rocblas_int>(nn);
    w.c = reduce ? cv.take<float>(nn * d) : nullptr;
    w.lib = cv.take<char>(lib_bytes);
    w.lib_bytes = lib_bytes;
    if (bytes) *bytes = cv.bytes();
    return w;
}

// factor blocks from the SVD: U'_K copied (its first K columns are contiguous, ld B), the first K
// rows of V'^T (column-major r x A, ld r) scaled by S into ld K:  blk_v[k + i K] = s[k] * vt[k + i r]
__global__ void k_rk_pack(const float* __restrict__ u, const float* __restrict__ vt, const float* __restrict__ s,
                          RkShape sh, int64_t n, float* __restrict__ blk, int64_t bstride) {
    const int64_t pu = sh.B * sh.K, pv = sh.K * sh.A, per = pu + pv, uo = rk_uoff(sh);
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n * per; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = t / per, q = t - b * per;
        float* dst = blk + b * bstride;
        if (q < pu) {
            dst[q] = u[b * sh.B * sh.r + q];
        } else {
            const int64_t z = q - pu, i = z / sh.K, k = z - i * sh.K;
            dst[uo + z] = s[b * sh.r + k] * vt[b * sh.r * sh.A + k + i * sh.r];
        }
    }
}

// gather n rows (any RowSrc) into a dense [n][d] matrix
__global__ void k_rk_gather(RowSrc rows, int64_t n, int64_t d, float* __restrict__ m) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n * d; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = t / d;
        m[t] = rows.row(i)[t - i * d];
    }
}

#define FLC_CHECK_RB(expr)                                                                     \
    do {                                                                                       \
        rocblas_status _s = (expr);                                                            \
        if (_s != rocblas_status_success) {                                                    \
            set_error("%s: rocBLAS/rocSOLVER status %d", #expr, (int)_s);                      \
            return FLC_ERR_HIP;                                                                \
        }                                                                                      \
    } while (0)

static rocblas_status rk_svd(rocblas_handle h, const RkShape& sh, int64_t n, float* m, float* s, float* u, float* vt,
                             float* e, rocblas_int* info) {
    const rocblas_int B = (rocblas_int)sh.B, A = (rocblas_int)sh.A, r = (rocblas_int)sh.r;
    return rocsolver_sgesvd_strided_batched(h, rocblas_svect_singular, rocblas_svect_singular, B, A, m, B,
                                            (rocblas_stride)sh.A * sh.B, s, r, u, B, (rocblas_stride)sh.B * sh.r, vt,
                                            r, (rocblas_stride)sh.r * sh.A, e, r, rocblas_outofplace, info,
                                            (rocblas_int)n);
}

// C_b (B x A, ld B: the row-major A x B result) = U'_K (S V'^T)_K from factor blocks bstride floats apart
static rocblas_status rk_gemm(rocblas_handle h, const RkShape& sh, int64_t n, const float* blk, int64_t bstride,
                              float* c) {
    const float one = 1.f, zero = 0.f;
    return rocblas_sgemm_strided_batched(h, rocblas_operation_none, rocblas_operation_none, (rocblas_int)sh.B,
                                         (rocblas_int)sh.A, (rocblas_int)sh.K, &one, blk, (rocblas_int)sh.B,
                                         (rocblas_stride)bstride, blk ? blk + rk_uoff(sh) : nullptr,
                                         (rocblas_int)sh.K, (rocblas_stride)bstride, &zero, c, (rocblas_int)sh.B,
                                         (rocblas_stride)sh.A * sh.B, (rocblas_int)n);
}

// device memory the library calls of one run need (the handle's size-query mode records it)
static size_t rk_lib_bytes_locked(rocblas_handle h, const RkShape& sh, int64_t n) {
    size_t sz = 0;
    if (rocblas_start_device_memory_size_query(h) != rocblas_status_success) return 0;
    (void)rk_svd(h, sh, n, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr);
    if (sh.K > 0) (void)rk_gemm(h, sh, n, nullptr, rk_block(sh), nullptr);
    if (rocblas_stop_device_memory_size_query(h, &sz) != rocblas_status_success) return 0;
    return sz;
}

size_t rk_workspace(const flc_codec_params* prm, int64_t n, int64_t d, bool reduce) {
    if (d < 1 || n < 1) return 0;
    const RkShape sh = rk_shape(d, prm->k);
    size_t lib = 0;
    {
        std::lock_guard<std::mutex> lk(g_rk_mu);
        rocblas_handle h = rk_handle();
        if (h) lib = rk_lib_bytes_locked(h, sh, n);
    }
    size_t b = 0;
    carve_rk(nullptr, sh, n, d, reduce, lib, &b);
    return b;
}

int rk_run(const flc_codec_params* prm, RowSrc rows, int64_t n, int64_t d, bool reduce, const float* w, float wt,
           float* out, void* wsp, size_t ws_bytes, hipStream_t st) {
    if (d == 0 || n == 0) return FLC_OK;
    if (prm->k < 1) { set_error("rank_k: K=%lld < 1", (long long)prm->k); return FLC_ERR_ARG; }
    if (d >= (int64_t)0x7FFFFFFF) { set_error("rank_k: D too large for rocSOLVER's 32-bit sizes"); return FLC_ERR_ARG; }
    const RkShape sh = rk_shape(d, prm->k);
    std::lock_guard<std::mutex> lk(g_rk_mu);
    rocblas_handle h = rk_handle();
    if (!h) { set_error("rank_k: rocblas_create_handle failed"); return FLC_ERR_HIP; }
    const size_t lib = rk_lib_bytes_locked(h, sh, n);
    size_t need = 0;
    carve_rk(nullptr, sh, n, d, reduce, lib, &need);
    if (ws_bytes < need) { set_error("rank_k: workspace %zu < %zu", ws_bytes, need); return FLC_ERR_WORKSPACE; }
    RkWs ws = carve_rk(wsp, sh, n, d, reduce, lib, nullptr);
    FLC_CHECK_RB(rocblas_set_stream(h, st));
    FLC_CHECK_RB(rocblas_set_workspace(h, ws.lib, ws.lib_bytes));
    float* c = reduce ? ws.c : out;
    const int gb = (int)std::max<int64_t>(1, std::min<int64_t>((n * d + 255) / 256, 4096));
    hipLaunchKernelGGL(k_rk_gather, dim3(gb), dim3(256), 0, st, rows, n, d, ws.m);
    FLC_CHECK_LAUNCH("k_rk_gather");
    FLC_CHECK_RB(rk_svd(h, sh, n, ws.m, ws.s, ws.u, ws.vt, ws.e, ws.info));
    if (sh.K > 0) {
        const int gs = (int)std::max<int64_t>(1, std::min<int64_t>((n * rk_block(sh) + 255) / 256, 4096));
        hipLaunchKernelGGL(k_rk_pack, dim3(gs), dim3(256), 0, st, ws.u, ws.vt, ws.s, sh, n, ws.blk, rk_block(sh));
        FLC_CHECK_LAUNCH("k_rk_pack");
        FLC_CHECK_RB(rk_gemm(h, sh, n, ws.blk, rk_block(sh), c));
    } else {
        FLC_CHECK_HIP(hipMemsetAsync(c, 0, (size_t)n * d * sizeof(float), st));
    }
    FLC_CHECK_RB(rocblas_set_workspace(h, nullptr, 0));
    if (!reduce) return FLC_OK;
    RowSrc cr{c, d, nullptr};
    return reduce_impl(cr, (d % 4) == 0, n, d, nullptr, w, wt, FLC_REDUCE_PLAIN, out, st);
}

// ---- wire format (wire.hip FMT_RANKK): the payload body is one row's factor block ----------------
int64_t rk_payload_floats(const flc_codec_params* prm, int64_t d) { return rk_block(rk_shape(d, prm->k)); }
int64_t rk_rank(const flc_codec_params* prm, int64_t d) { return rk_shape(d, prm->k).K; }

__global__ void k_rk_gather_blocks(const char* __restrict__ base, int64_t ld, const char* const* __restrict__ ptrs,
                                   int64_t n, int64_t per, float* __restrict__ blk) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n * per; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = t / per, q = t - b * per;
        const float* src = reinterpret_cast<const float*>((base ? base + b * ld : ptrs[b]) + 16);
        blk[t] = src[q];
    }
}

int rk_pack(const flc_codec_params* prm, const float* x, int64_t d, float* body, void* wsp, size_t ws_bytes,
            hipStream_t st) {
    if (prm->k < 1) { set_error("rank_k: K=%lld < 1", (long long)prm->k); return FLC_ERR_ARG; }
    if (d >= (int64_t)0x7FFFFFFF) { set_error("rank_k: D too large for rocSOLVER's 32-bit sizes"); return FLC_ERR_ARG; }
    const RkShape sh = rk_shape(d, prm->k);
    std::lock_guard<std::mutex> lk(g_rk_mu);
    rocblas_handle h = rk_handle();
    if (!h) { set_error("rank_k: rocblas_create_handle failed"); return FLC_ERR_HIP; }
    const size_t lib = rk_lib_bytes_locked(h, sh, 1);
    size_t need = 0;
    carve_rk(nullptr, sh, 1, d, false, lib, &need);
    if (ws_bytes < need) { set_error("rank_k pack: workspace %zu < %zu", ws_bytes, need); return FLC_ERR_WORKSPACE; }
    RkWs ws = carve_rk(wsp, sh, 1, d, false, lib, nullptr);
    FLC_CHECK_RB(rocblas_set_stream(h, st));
    FLC_CHECK_RB(rocblas_set_workspace(h, ws.lib, ws.lib_bytes));
    RowSrc r{x, d, nullptr};
    const int gb = (int)std::max<int64_t>(1, std::min<int64_t>((d + 255) / 256, 4096));
    hipLaunchKernelGGL(k_rk_gather, dim3(gb), dim3(256), 0, st, r, (int64_t)1, d, ws.m);
    FLC_CHECK_LAUNCH("k_rk_gather");
    FLC_CHECK_RB(rk_svd(h, sh, 1, ws.m, ws.s, ws.u, ws.vt, ws.e, ws.info));
    if (sh.K > 0) {
        const int gs = (int)std::max<int64_t>(1, std::min<int64_t>((rk_block(sh) + 255) / 256, 4096));
        hipLaunchKernelGGL(k_rk_pack, dim3(gs), dim3(256), 0, st, ws.u, ws.vt, ws.s, sh, (int64_t)1, body, rk_block(sh));
        FLC_CHECK_LAUNCH("k_rk_pack");
    }
    FLC_CHECK_RB(rocblas_set_workspace(h, nullptr, 0));
    return FLC_OK;
}

// one payload decoded in place of the row (flc_unpack has no workspace: rocBLAS's own device memory)
int rk_unpack1(const flc_codec_params* prm, const float* body, int64_t d, float* out, hipStream_t st) {
    if (d == 0) return FLC_OK;
    const RkShape sh = rk_shape(d, prm->k);
    if (sh.K == 0) { FLC_CHECK_HIP(hipMemsetAsync(out, 0, (size_t)d * sizeof(float), st)); return FLC_OK; }
    std::lock_guard<std::mutex> lk(g_rk_mu);
    rocblas_handle h = rk_handle();
    if (!h) { set_error("rank_k: rocblas_create_handle failed"); return FLC_ERR_HIP; }
    FLC_CHECK_RB(rocblas_set_stream(h, st));
    FLC_CHECK_RB(rocblas_set_workspace(h, nullptr, 0));
    FLC_CHECK_RB(rk_gemm(h, sh, 1, body, rk_block(sh), out));
    return FLC_OK;
}

size_t rk_unpack_workspace(const flc_codec_params* prm, int64_t n, int64_t d) {
    if (d < 1 || n < 1) return 0;
    const RkShape sh = rk_shape(d, prm->k);
    size_t lib = 0;
    {
        std::lock_guard<std::mutex> lk(g_rk_mu);
        rocblas_handle h = rk_handle();
        if (h && rocblas_start_device_memory_size_query(h) == rocblas_status_success) {
            if (sh.K > 0) (void)rk_gemm(h, sh, n, nullptr, rk_block(sh), nullptr);
            (void)rocblas_stop_device_memory_size_query(h, &lib);
        }
    }
    Carver cv(nullptr);
    cv.take<float>((size_t)n * std::max<int64_t>(rk_block(sh), 1));
    cv.take<float>((size_t)n * d);
    cv.take<char>(lib);
    return cv.bytes();
}

// n payloads -> factor blocks in the workspace -> the encode's GEMM -> the fold (n == 1 and out:
// the decode itself, written straight to out)
int rk_unpack_reduce(const flc_codec_params* prm, const char* base, int64_t ld, const char* const* ptrs, int64_t n,
                     int64_t d, const float* w, float wt, float* out, bool reduce, void* wsp, size_t ws_bytes,
                     hipStream_t st) {
    if (d == 0 || n == 0) return FLC_OK;
    const RkShape sh = rk_shape(d, prm->k);
    const size_t need = rk_unpack_workspace(prm, n, d);
    if (ws_bytes < need) { set_error("rank_k unpack: workspace %zu < %zu", ws_bytes, need); return FLC_ERR_WORKSPACE; }
    Carver cv(wsp);
    float* blk = cv.take<float>((size_t)n * std::max<int64_t>(rk_block(sh), 1));
    float* c = cv.take<float>((size_t)n * d);
    const size_t lib = need - cv.bytes();
    void* libp = cv.take<char>(lib);
    std::lock_guard<std::mutex> lk(g_rk_mu);
    rocblas_handle h = rk_handle();
    if (!h) { set_error("rank_k: rocblas_create_handle failed"); return FLC_ERR_HIP; }
    FLC_CHECK_RB(rocblas_set_stream(h, st));
    FLC_CHECK_RB(rocblas_set_workspace(h, libp, lib));
    float* dst = reduce ? c : out;
    if (sh.K > 0) {
        const int gs = (int)std::max<int64_t>(1, std::min<int64_t>((n * rk_block(sh) + 255) / 256, 4096));
        hipLaunchKernelGGL(k_rk_gather_blocks, dim3(gs), dim3(256), 0, st, base, ld, ptrs, n, rk_block(sh), blk);
        FLC_CHECK_LAUNCH("k_rk_gather_blocks");
        FLC_CHECK_RB(rk_gemm(h, sh, n, blk, rk_block(sh), dst));
    } else {
        FLC_CHECK_HIP(hipMemsetAsync(dst, 0, (size_t)n * d * sizeof(float), st));
    }
    FLC_CHECK_RB(rocblas_set_workspace(h, nullptr, 0));
    if (!reduce) return FLC_OK;
    RowSrc cr{c, d, nullptr};
    return reduce_impl(cr, (d % 4) == 0, n, d, nullptr, w, wt, FLC_REDUCE_PLAIN, out, st);
}

}  // namespace flc
