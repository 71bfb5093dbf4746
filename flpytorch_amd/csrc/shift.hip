// Shift codecs: the client-side update of the compressed algorithms,
//     e = C(a - b);   msg = base + e * scale;   h_out = h_in + alpha * e
// DIANA  m_i = C(g - h_i), h_i += alpha m_i                      algorithms.py:1383-1391
// EF21   g_next = g_prev + C(g - g_prev) * (1 / (1 + w) | 1)     algorithms.py:1506-1517
// MARINA g_next = g_prev + C(g - g_prev_x)                       algorithms.py:537, 691
// FRECON / COFIG u_i = C(g - h_i), h_i += alpha u_i              algorithms.py:1104-1110, 1265-1269
//
// Elementwise codecs (ident, lazy, natural, dithering) run one fused pass (codecs.hip k_ew_shift,
// after the norm pass over a - b for dithering): a, b [, base, h_in] read once, msg [, h_out]
// written once, e never stored.  RandK / TopK / Rank-K select or factor the whole difference first:
// a - b is formed once in the workspace, encoded by the ordinary single-row path into a second
// workspace row, and k_shift_epi applies the same epilogue.
#include "common.hpp"

namespace flc {

__global__ __launch_bounds__(256) void k_shift_sub(const float* __restrict__ a, const float* __restrict__ b, int64_t d,
                                                   float* __restrict__ diff) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t g4 = d / 4;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < g4; g += stride) {
        const float4 x = reinterpret_cast<const float4*>(a)[g], y = reinterpret_cast<const float4*>(b)[g];
        reinterpret_cast<float4*>(diff)[g] = make_float4(x.x - y.x, x.y - y.y, x.z - y.z, x.w - y.w);
    }
    for (int64_t j = g4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += stride) diff[j] = a[j] - b[j];
}

__global__ __launch_bounds__(256) void k_shift_sub_scalar(const float* __restrict__ a, const float* __restrict__ b,
                                                          int64_t d, float* __restrict__ diff) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += (int64_t)gridDim.x * blockDim.x)
        diff[j] = a[j] - b[j];
}

// the epilogue over a stored e (scalar loads: the caller's msg / base / h may be unaligned views)
__global__ __launch_bounds__(256) void k_shift_epi(const float* __restrict__ e, int64_t d, ShiftArgs sh) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += (int64_t)gridDim.x * blockDim.x) {
        const float v = e[j];
        if (sh.msg) {
            const float t = v * sh.scale;
            sh.msg[j] = sh.base ? sh.base[j] + t : t;
        }
        if (sh.hout) sh.hout[j] = sh.hin[j] + sh.alpha * v;
    }
}

static bool shift_elementwise(int codec) { return codec != FLC_RANDK && codec != FLC_TOPK && codec != FLC_RANK_K; }

static size_t inner_workspace(const flc_codec_params* prm, int64_t d) {
    if (prm->codec == FLC_TOPK) return sel_workspace(prm, 1, d);
    if (prm->codec == FLC_RANK_K) return rk_workspace(prm, 1, d, false);
    return randk_device_workspace(1, d);   // RandK: the device draws' chunk counts
}

size_t shift_workspace(const flc_codec_params* prm, int64_t d) {
    if (shift_elementwise(prm->codec)) return ew_workspace(prm, 1, d);
    Carver c(nullptr);
    c.take<float>((size_t)d);
    c.take<float>((size_t)d);
    c.take<char>(inner_workspace(prm, d));
    return c.bytes();
}

int shift_run(const flc_codec_params* prm, const flc_pattern* pat, const float* a, int64_t d, const ShiftArgs& sh,
              float* pnorm_out, void* ws, size_t ws_bytes, hipStream_t st) {
    if (d == 0) return FLC_OK;
    if (ws_bytes < shift_workspace(prm, d)) { set_error("flc_encode_shift: workspace too small"); return FLC_ERR_WORKSPACE; }
    if (shift_elementwise(prm->codec)) {
        const bool vec = (((uintptr_t)a | (uintptr_t)sh.b) & 15u) == 0;
        RowSrc s{a, d, nullptr};
        return ew_run(prm, pat, s, vec, 1, d, nullptr, pnorm_out, /*dense=*/true, nullptr, nullptr, 1.f, ws, ws_bytes,
                      st, &sh);
    }
    Carver c(ws);
    float* diff = c.take<float>((size_t)d);
    float* e = c.take<float>((size_t)d);
    const size_t inner = inner_workspace(prm, d);
    void* iws = c.take<char>(inner);
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((d + 1023) / 1024, 4096));
    if ((((uintptr_t)a | (uintptr_t)sh.b) & 15u) == 0)
        hipLaunchKernelGGL(k_shift_sub, dim3(grid), dim3(256), 0, st, a, sh.b, d, diff);
    else
        hipLaunchKernelGGL(k_shift_sub_scalar, dim3(grid), dim3(256), 0, st, a, sh.b, d, diff);
    FLC_CHECK_LAUNCH("k_shift_sub");
    int rc = FLC_OK;
    RowSrc r{diff, d, nullptr};
    if (prm->codec == FLC_RANDK) {
        if (!(pat && pat->d_randk_idx) && prm->k > d) { set_error("randk: K > D"); return FLC_ERR_ARG; }
        rc = randk_dense(prm, pat, diff, d, e, iws, inner, st);
    } else if (prm->codec == FLC_TOPK) {
        rc = sel_run(prm, pat, r, true, 1, d, /*assign=*/true, nullptr, 1.f, e, iws, inner, st);
    } else {
        rc = rk_run(prm, r, 1, d, /*reduce=*/false, nullptr, 1.f, e, iws, inner, st);
    }
    if (rc) return rc;
    const int g2 = (int)std::max<int64_t>(1, std::min<int64_t>((d + 255) / 256, 8192));
    hipLaunchKernelGGL(k_shift_epi, dim3(g2), dim3(256), 0, st, e, d, sh);
    FLC_CHECK_LAUNCH("k_shift_epi");
    return FLC_OK;
}

}  // namespace flc
