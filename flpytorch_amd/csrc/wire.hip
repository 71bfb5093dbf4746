// Wire format: the compressed message a client would actually send, and the
// server's decode + reduce straight from the N messages (fl_pytorch/utils/compressors.py:223-224,
// 367-368 count these bits as last_need_to_send_advance, but the reference only ever moves the
// dense decoded tensor; comm_socket.py pickles that).
//
// One row's payload: a 16-B header {u32 format, u32 count, f32 norm, u32 bad} and a body, 16-B padded:
//   F32     ident / lazy / natural dithering (the reference's output is ~x): f32[d]
//   Q8      standard dithering / QSGD / TernGrad, s <= 127: u8[d]   bit 7 sign, bits 0-6 level index
//   Q16     standard dithering, 127 < s <= 32767:         u16[d]  bit 15 sign, bits 0-14 level index
//   NAT16   natural:                                       u16[d]  bit 15 sign, bits 0-14: 0 zero,
//           0x7FFE inf, 0x7FFF NaN, else k + 16384 for the value 2^k (k in [-149, 127])
//   SPARSE  randk / topk: count (<= K) entries, u32 idx[K] then f32 val[K], ascending idx; the
//           entries are the output's elements whose bits are not +0
//   RANKK   rank_k: the factor block of rank_k.hip — U'_K (B x K) then (S V'^T)_K (K x A), f32,
//           K' (A + B) values as the reference counts them (compressors.py:362)
// Level codes: value = (levels[idx] * sign) * norm exactly as the encode (compressors.py:294-296);
// code 0 is +0 exactly (x == 0), sign + level 0 with the sign bit is -0 * norm (NaN when the norm is
// not finite).  Decoding a payload gives the dense compressVector output bit for bit
// (flc_pack -> flc_unpack), and flc_unpack_reduce equals flc_encode_reduce of the same rows.
//
// flc_pack runs the row's ordinary encode into the workspace first (so every draw, norm and tie
// rule is the encode's) and derives the codes from the dense output: a level index is the one whose
// (levels[i] * sign) * norm reproduces the element's bits (guess rint(y s), then its neighbours,
// then a binary search); elements no level reproduces are counted in the header's `bad` field
// (never seen: the encode's outputs are of that form by construction; the tests assert 0).
#include <cstring>

#include "wire_codes.hpp"

namespace flc {

int payload_format(const flc_codec_params* prm) {
    switch (prm->codec) {
        case FLC_STD_DITHERING: return prm->s <= 127 ? FMT_Q8 : FMT_Q16;
        case FLC_NATURAL: return FMT_NAT16;
        case FLC_RANDK:
        case FLC_TOPK: return FMT_SPARSE;
        case FLC_RANK_K: return FMT_RANKK;
        default: return FMT_F32;
    }
}

int64_t payload_bytes(const flc_codec_params* prm, int64_t d) {
    switch (payload_format(prm)) {
        case FMT_Q8: return 16 + a16(d);
        case FMT_Q16:
        case FMT_NAT16: return 16 + a16(2 * d);
        case FMT_SPARSE: { const int64_t k = std::max<int64_t>(1, std::min(prm->k, d)); return 16 + 2 * a16(4 * k); }
        case FMT_RANKK: return 16 + a16(4 * rk_payload_floats(prm, d));
        default: return 16 + a16(4 * d);
    }
}

// ---- pack ---------------------------------------------------------------------------------------
__global__ void k_rankk_header(char* payload, uint32_t floats, uint32_t k) {
    if (threadIdx.x == 0) {
        PayloadHeader* h = reinterpret_cast<PayloadHeader*>(payload);
        h->fmt = FMT_RANKK;
        h->count = k;          // rank of the expansion (K' = min(K, A, B) factors are stored)
        h->norm = 0.f;
        h->bad = 0u;
        (void)floats;
    }
}

__global__ __launch_bounds__(256) void k_pack_dense(const float* __restrict__ v, int64_t d, int fmt,
                                                    const float* __restrict__ levels, int s,
                                                    const float* __restrict__ pnorm, char* __restrict__ payload) {
    PayloadHeader* h = reinterpret_cast<PayloadHeader*>(payload);
    char* body = payload + 16;
    const float norm = pnorm ? *pnorm : 0.f;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        h->fmt = (uint32_t)fmt;
        h->count = (uint32_t)d;
        h->norm = norm;
    }
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += (int64_t)gridDim.x * blockDim.x) {
        const float x = v[j];
        if (fmt == FMT_F32) reinterpret_cast<float*>(body)[j] = x;
        else if (fmt == FMT_Q8) reinterpret_cast<uint8_t*>(body)[j] = (uint8_t)lev_code(x, levels, s, norm, 0x80u, &h->bad);
        else if (fmt == FMT_Q16) reinterpret_cast<uint16_t*>(body)[j] = (uint16_t)lev_code(x, levels, s, norm, 0x8000u, &h->bad);
        else reinterpret_cast<uint16_t*>(body)[j] = (uint16_t)nat_code(x);
    }
}

__global__ void k_pack_header(char* payload, uint32_t fmt, uint32_t count) {
    if (threadIdx.x == 0) {
        PayloadHeader* h = reinterpret_cast<PayloadHeader*>(payload);
        h->fmt = fmt;
        h->count = count;
        h->norm = 0.f;
        h->bad = 0u;
    }
}

constexpr int PK_BLK = 4096;   // elements per compaction block

__global__ __launch_bounds__(256) void k_pack_count(const float* __restrict__ v, int64_t d, uint32_t* __restrict__ bc) {
    const int64_t b = blockIdx.x, j0 = b * PK_BLK, j1 = min(d, j0 + PK_BLK);
    uint32_t c = 0;
    for (int64_t j = j0 + threadIdx.x; j < j1; j += 256) c += __float_as_uint(v[j]) != 0u;
    c = wave_sum(c);
    __shared__ uint32_t ws4[4];
    if ((threadIdx.x & 63) == 0) ws4[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) bc[b] = ws4[0] + ws4[1] + ws4[2] + ws4[3];
}

__global__ __launch_bounds__(1024) void k_pack_scan(uint32_t* __restrict__ bc, int64_t nb, char* __restrict__ payload,
                                                    int64_t cap) {
    __shared__ uint32_t wsum[16];
    const int tid = threadIdx.x;
    const int64_t per = (nb + 1023) / 1024, q0 = min<int64_t>(nb, tid * per), q1 = min<int64_t>(nb, q0 + per);
    uint32_t loc = 0;
    for (int64_t q = q0; q < q1; ++q) loc += bc[q];
    uint32_t incl = loc;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(incl, o, WAVE);
        if ((tid & 63) >= o) incl += u;
    }
    if ((tid & 63) == 63) wsum[tid >> 6] = incl;
    __syncthreads();
    uint32_t run = incl - loc;
    for (int w = 0; w < (tid >> 6); ++w) run += wsum[w];
    for (int64_t q = q0; q < q1; ++q) { const uint32_t c = bc[q]; bc[q] = run; run += c; }
    if (tid == 1023) {
        PayloadHeader* h = reinterpret_cast<PayloadHeader*>(payload);
        h->fmt = FMT_SPARSE;
        h->count = run;
        h->norm = 0.f;
        h->bad = run > (uint64_t)cap ? run - (uint32_t)cap : 0u;   // more nonzeros than K: never for RandK / TopK
    }
}

__global__ __launch_bounds__(256) void k_pack_write(const float* __restrict__ v, int64_t d, const uint32_t* __restrict__ bc,
                                                    char* __restrict__ payload, int64_t cap) {
    const int64_t b = blockIdx.x, j0 = b * PK_BLK;
    uint32_t* idx = reinterpret_cast<uint32_t*>(payload + 16);
    float* val = reinterpret_cast<float*>(payload + 16 + a16(4 * cap));
    __shared__ uint32_t wsum[4];
    uint32_t base = bc[b];
    for (int64_t s0 = j0; s0 < min(d, j0 + PK_BLK); s0 += 256) {
        const int64_t j = s0 + threadIdx.x;
        const float x = j < d ? v[j] : 0.f;
        const bool keep = j < d && __float_as_uint(x) != 0u;
        const uint64_t m = __ballot(keep);
        const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (lane == 0) wsum[wv] = (uint32_t)__builtin_popcountll(m);
        __syncthreads();
        uint32_t off = base;
        for (uint32_t w = 0; w < wv; ++w) off += wsum[w];
        if (keep && off + rank < (uint64_t)cap) { idx[off + rank] = (uint32_t)j; val[off + rank] = x; }
        base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();
    }
}

// ---- unpack (one row) --------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_unpack_dense(const char* __restrict__ payload, int64_t d, int fmt, int s,
                                                      const float* __restrict__ levels, float* __restrict__ out) {
    // the format and level count come from the codec, never from the message: a header that lies
    // cannot move a read past the body flc_payload_bytes sized (flc_payload_validate reports it)
    const float norm = reinterpret_cast<const PayloadHeader*>(payload)->norm;
    const char* body = payload + 16;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += (int64_t)gridDim.x * blockDim.x) {
        float x;
        if (fmt == FMT_F32) x = reinterpret_cast<const float*>(body)[j];
        else if (fmt == FMT_Q8) x = lev_decode(reinterpret_cast<const uint8_t*>(body)[j], levels, s, norm, 0x80u);
        else if (fmt == FMT_Q16) x = lev_decode(reinterpret_cast<const uint16_t*>(body)[j], levels, s, norm, 0x8000u);
        else x = nat_decode(reinterpret_cast<const uint16_t*>(body)[j]);
        out[j] = x;
    }
}

__global__ __launch_bounds__(256) void k_unpack_sparse(const char* __restrict__ payload, int64_t cap, int64_t d,
                                                       float* __restrict__ out) {
    const PayloadHeader h = *reinterpret_cast<const PayloadHeader*>(payload);
    const uint32_t* idx = reinterpret_cast<const uint32_t*>(payload + 16);
    const float* val = reinterpret_cast<const float*>(payload + 16 + a16(4 * cap));
    const int64_t cnt = min<int64_t>(h.count, cap);
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < cnt; e += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t j = idx[e];
        if (j < (uint64_t)d) out[j] = val[e];                  // an index past the row is never written
    }
}

// ---- decode + reduce over n payloads (dense formats) --------------------------------------------
// Tile owner: each thread owns the E elements of one 16-B body slice (E = 16 Q8 codes, 8 Q16 /
// NAT16 codes, 4 floats) for the whole fold, rows in order, PF rows' slices in flight (a register
// ring), so the fp32 sum is the sequential one: acc = t_0; acc = acc + t_i; out = acc / wt with
// t_i = w_i * dec_i.  Q8 level tables (<= 128 levels) sit in LDS.
template <int FMT>
struct WireFmt {
    static constexpr int E = FMT == FMT_Q8 ? 16 : (FMT == FMT_F32 ? 4 : 8);
    static constexpr int BYTES = 16 / E;
};

template <int FMT>
__device__ inline float dec1(uint32_t c, const float* lv, int s, float norm) {
    if (FMT == FMT_Q8) return lev_decode(c, lv, s, norm, 0x80u);
    if (FMT == FMT_Q16) return lev_decode(c, lv, s, norm, 0x8000u);
    if (FMT == FMT_NAT16) return nat_decode(c);
    return __uint_as_float(c);
}

template <int FMT>
__device__ inline void dec16(uint4 v, const float* lv, int s, float norm, float* e) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    constexpr int E = WireFmt<FMT>::E;
#pragma unroll
    for (int q = 0; q < E; ++q) {
        uint32_t c;
        if (FMT == FMT_Q8) c = (w[q >> 2] >> (8 * (q & 3))) & 0xFFu;
        else if (FMT == FMT_F32) c = w[q];
        else c = (w[q >> 1] >> (16 * (q & 1))) & 0xFFFFu;
        e[q] = dec1<FMT>(c, lv, s, norm);
    }
}

template <int FMT, bool W, int PF>
__global__ __launch_bounds__(256) void k_unpack_accum(const char* __restrict__ base, int64_t ld,
                                                      const char* const* __restrict__ ptrs, int64_t n, int64_t d,
                                                      const float* __restrict__ levels, int s,
                                                      const float* __restrict__ w, float wt, float* __restrict__ out) {
    constexpr int E = WireFmt<FMT>::E;
    __shared__ float lvs[128];
    const float* lv = levels;
    if (FMT == FMT_Q8) {
        for (int i = threadIdx.x; i <= s && i < 128; i += 256) lvs[i] = levels[i];
        __syncthreads();
        lv = lvs;
    }
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t j0 = g * E;
    const int64_t full = d / E;                       // complete 16-B slices
    auto row = [&](int64_t i) -> const char* { return base ? base + i * ld : sload(ptrs + i); };
    if (g < full) {
        uint4 ring[PF];
#pragma unroll
        for (int p = 0; p < PF; ++p)
            if (p < n) ring[p] = *reinterpret_cast<const uint4*>(row(p) + 16 + g * 16);
        float acc[E];
        for (int64_t i0 = 0; i0 < n; i0 += PF) {
#pragma unroll
            for (int p = 0; p < PF; ++p) {
                const int64_t i = i0 + p;
                if (i < n) {
                    const char* r = row(i);
                    const float norm = (FMT == FMT_Q8 || FMT == FMT_Q16) ? sload(reinterpret_cast<const float*>(r + 8)) : 0.f;
                    const float wi = W ? w[i] : 1.f;
                    float e[E];
                    dec16<FMT>(ring[p], lv, s, norm, e);
                    if (i + PF < n) ring[p] = *reinterpret_cast<const uint4*>(row(i + PF) + 16 + g * 16);
#pragma unroll
                    for (int q = 0; q < E; ++q) {
                        const float t = W ? wi * e[q] : e[q];
                        acc[q] = (i == 0) ? t : acc[q] + t;
                    }
                }
            }
        }
        float4* o4 = reinterpret_cast<float4*>(out + j0);
        if (((uintptr_t)(out + j0) & 15u) == 0) {
#pragma unroll
            for (int q = 0; q < E; q += 4) o4[q / 4] = make_float4(acc[q] / wt, acc[q + 1] / wt, acc[q + 2] / wt, acc[q + 3] / wt);
        } else {
#pragma unroll
            for (int q = 0; q < E; ++q) out[j0 + q] = acc[q] / wt;
        }
        return;
    }
    if (g == full && full * E < d) {                   // the tail: fewer than E elements, element loads
        const int m = (int)(d - full * E);
        float acc[E];
        for (int64_t i = 0; i < n; ++i) {
            const char* r = row(i);
            const float norm = (FMT == FMT_Q8 || FMT == FMT_Q16) ? reinterpret_cast<const float*>(r + 8)[0] : 0.f;
            const float wi = W ? w[i] : 1.f;
            for (int q = 0; q < m; ++q) {
                const int64_t j = full * E + q;
                uint32_t c;
                if (FMT == FMT_Q8) c = reinterpret_cast<const uint8_t*>(r + 16)[j];
                else if (FMT == FMT_F32) c = reinterpret_cast<const uint32_t*>(r + 16)[j];
                else c = reinterpret_cast<const uint16_t*>(r + 16)[j];
                const float e = dec1<FMT>(c, lv, s, norm);
                const float t = W ? wi * e : e;
                acc[q] = (i == 0) ? t : acc[q] + t;
            }
        }
        for (int q = 0; q < m; ++q) out[full * E + q] = acc[q] / wt;
    }
}

// ---- host ----------------------------------------------------------------------------------------
struct PackWs {
    float* dense;
    float* pnorm;
    uint32_t* bc;
    void* inner;
    size_t inner_bytes;
};
static PackWs carve_pack(void* base, const flc_codec_params* prm, int64_t d, size_t* bytes) {
    Carver c(base);
    PackWs w;
    w.dense = c.take<float>((size_t)std::max<int64_t>(d, 1));
    w.pnorm = c.take<float>(1);
    w.bc = c.take<uint32_t>((size_t)std::max<int64_t>((d + PK_BLK - 1) / PK_BLK, 1));
    w.inner_bytes = encode_row_workspace(prm, d);
    w.inner = c.take<char>(w.inner_bytes);
    if (bytes) *bytes = c.bytes();
    return w;
}

size_t pack_workspace(const flc_codec_params* prm, int64_t d) {
    if (payload_format(prm) == FMT_RANKK) return rk_workspace(prm, 1, d, false);
    size_t b = 0;
    carve_pack(nullptr, prm, d, &b);
    return b;
}

static bool natbug(const flc_codec_params* prm) { return prm->codec == FLC_NAT_DITHERING; }

int pack_run(const flc_codec_params* prm, const flc_pattern* pat, const float* x, int64_t d, char* payload, void* ws,
             size_t ws_bytes, hipStream_t st) {
    if (ws_bytes < pack_workspace(prm, d)) { set_error("flc_pack: workspace too small"); return FLC_ERR_WORKSPACE; }
    if ((uintptr_t)payload & 15u) { set_error("flc_pack: payload must be 16-byte aligned"); return FLC_ERR_ARG; }
    const int fmt = payload_format(prm);
    if (fmt == FMT_RANKK) {
        const int64_t pb = payload_bytes(prm, d);
        FLC_CHECK_HIP(hipMemsetAsync(payload, 0, (size_t)pb, st));
        if (d == 0) return FLC_OK;
        hipLaunchKernelGGL(k_rankk_header, dim3(1), dim3(64), 0, st, payload, (uint32_t)rk_payload_floats(prm, d),
                           (uint32_t)rk_rank(prm, d));
        FLC_CHECK_LAUNCH("k_rankk_header");
        return rk_pack(prm, x, d, reinterpret_cast<float*>(payload + 16), ws, ws_bytes, st);
    }
    PackWs w = carve_pack(ws, prm, d, nullptr);
    // header zeroed; the body's 16-B padding (and the unused part of a sparse list) zeroed too, so
    // a payload's bytes are a function of the row alone
    const int64_t pb = payload_bytes(prm, d);
    if (fmt == FMT_SPARSE) FLC_CHECK_HIP(hipMemsetAsync(payload, 0, (size_t)pb, st));
    else {
        FLC_CHECK_HIP(hipMemsetAsync(payload, 0, 16, st));
        FLC_CHECK_HIP(hipMemsetAsync(payload + pb - 16, 0, 16, st));
    }
    if (d == 0) {
        // header {fmt, 0, 0, 0} written by a kernel: no host staging, no synchronisation
        hipLaunchKernelGGL(k_pack_header, dim3(1), dim3(64), 0, st, payload, (uint32_t)fmt, 0u);
        FLC_CHECK_LAUNCH("k_pack_header");
        return FLC_OK;
    }
    const bool dither = fmt == FMT_Q8 || fmt == FMT_Q16;
    if (dither || fmt == FMT_NAT16) {
        // one pass: the encode writes its codes straight into the payload (codecs.hip k_ew_code)
        CodeArgs ca{fmt, payload, prm->d_levels, prm->s, dither ? w.pnorm : nullptr};
        RowSrc src{x, d, nullptr};
        return ew_run(prm, pat, src, ((uintptr_t)x & 15u) == 0, 1, d, nullptr, dither ? w.pnorm : nullptr,
                      /*dense=*/true, nullptr, nullptr, 1.f, w.inner, w.inner_bytes, st, nullptr, &ca);
    }
    if (fmt == FMT_F32) {
        // the dense encode written straight into the body, then the header
        int rc = encode_row(prm, pat, x, d, nullptr, nullptr, reinterpret_cast<float*>(payload + 16), w.inner,
                            w.inner_bytes, st);
        if (rc) return rc;
        hipLaunchKernelGGL(k_pack_header, dim3(1), dim3(64), 0, st, payload, (uint32_t)fmt, (uint32_t)d);
        FLC_CHECK_LAUNCH("k_pack_header");
        return FLC_OK;
    }
    int rc = encode_row(prm, pat, x, d, nullptr, dither ? w.pnorm : nullptr, w.dense, w.inner, w.inner_bytes, st);
    if (rc) return rc;
    (void)natbug;
    if (fmt == FMT_SPARSE) {
        const int64_t nb = (d + PK_BLK - 1) / PK_BLK, cap = std::max<int64_t>(1, std::min(prm->k, d));
        hipLaunchKernelGGL(k_pack_count, dim3((unsigned)nb), dim3(256), 0, st, w.dense, d, w.bc);
        FLC_CHECK_LAUNCH("k_pack_count");
        hipLaunchKernelGGL(k_pack_scan, dim3(1), dim3(1024), 0, st, w.bc, nb, payload, cap);
        FLC_CHECK_LAUNCH("k_pack_scan");
        hipLaunchKernelGGL(k_pack_write, dim3((unsigned)nb), dim3(256), 0, st, w.dense, d, w.bc, payload, cap);
        FLC_CHECK_LAUNCH("k_pack_write");
        return FLC_OK;
    }
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((d + 255) / 256, 8192));
    hipLaunchKernelGGL(k_pack_dense, dim3(grid), dim3(256), 0, st, w.dense, d, fmt, prm->d_levels, prm->s,
                       dither ? w.pnorm : nullptr, payload);
    FLC_CHECK_LAUNCH("k_pack_dense");
    return FLC_OK;
}

int unpack_run(const flc_codec_params* prm, const char* payload, int64_t d, float* out, hipStream_t st) {
    if (d == 0) return FLC_OK;
    if ((uintptr_t)payload & 15u) { set_error("flc_unpack: payload must be 16-byte aligned"); return FLC_ERR_ARG; }
    const int fmt = payload_format(prm);
    if (fmt == FMT_RANKK) return rk_unpack1(prm, reinterpret_cast<const float*>(payload + 16), d, out, st);
    if (fmt == FMT_SPARSE) {
        const int64_t cap = std::max<int64_t>(1, std::min(prm->k, d));
        FLC_CHECK_HIP(hipMemsetAsync(out, 0, (size_t)d * sizeof(float), st));
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((cap + 255) / 256, 4096));
        hipLaunchKernelGGL(k_unpack_sparse, dim3(grid), dim3(256), 0, st, payload, cap, d, out);
        FLC_CHECK_LAUNCH("k_unpack_sparse");
        return FLC_OK;
    }
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((d + 255) / 256, 8192));
    hipLaunchKernelGGL(k_unpack_dense, dim3(grid), dim3(256), 0, st, payload, d, fmt, prm->s, prm->d_levels, out);
    FLC_CHECK_LAUNCH("k_unpack_dense");
    return FLC_OK;
}

// Host check of one message as it comes off the network (flc_payload_validate): everything the
// decode kernels take from the message itself — header format, count, the level codes, the sparse
// indices — against what the codec and d allow.
int payload_validate(const flc_codec_params* prm, const uint8_t* p, int64_t nbytes, int64_t d) {
    const int64_t pb = payload_bytes(prm, d);
    if (nbytes < pb) { set_error("payload: %lld bytes, the message of d=%lld is %lld", (long long)nbytes, (long long)d, (long long)pb); return FLC_ERR_ARG; }
    if (d == 0) return FLC_OK;
    PayloadHeader h;
    std::memcpy(&h, p, sizeof h);
    const int fmt = payload_format(prm);
    if ((int)h.fmt != fmt) { set_error("payload: header format %u, the codec's is %d", h.fmt, fmt); return FLC_ERR_ARG; }
    if (h.bad != 0u) { set_error("payload: %u elements flagged unrepresentable by the sender", h.bad); return FLC_ERR_ARG; }
    const uint8_t* body = p + 16;
    switch (fmt) {
        case FMT_Q8:
        case FMT_Q16: {
            if (h.count != (uint32_t)d) { set_error("payload: count %u != d", h.count); return FLC_ERR_ARG; }
            const uint32_t mask = fmt == FMT_Q8 ? 0x7Fu : 0x7FFFu;
            for (int64_t j = 0; j < d; ++j) {
                uint32_t c;
                if (fmt == FMT_Q8) c = body[j];
                else { uint16_t v; std::memcpy(&v, body + 2 * j, 2); c = v; }
                if ((c & mask) > (uint32_t)prm->s) { set_error("payload: level code %u at %lld exceeds s=%d", c & mask, (long long)j, prm->s); return FLC_ERR_ARG; }
            }
            return FLC_OK;
        }
        case FMT_F32:
        case FMT_NAT16:
            if (h.count != (uint32_t)d) { set_error("payload: count %u != d", h.count); return FLC_ERR_ARG; }
            return FLC_OK;
        case FMT_SPARSE: {
            const int64_t cap = std::max<int64_t>(1, std::min(prm->k, d));
            if ((int64_t)h.count > cap) { set_error("payload: %u entries, at most K=%lld", h.count, (long long)cap); return FLC_ERR_ARG; }
            int64_t prev = -1;
            for (uint32_t e = 0; e < h.count; ++e) {
                uint32_t j;
                std::memcpy(&j, body + 4 * (int64_t)e, 4);
                if ((int64_t)j >= d || (int64_t)j <= prev) { set_error("payload: entry %u index %u not ascending in [0, d)", e, j); return FLC_ERR_ARG; }
                prev = j;
            }
            return FLC_OK;
        }
        case FMT_RANKK:
            if ((int64_t)h.count != rk_rank(prm, d)) { set_error("payload: rank %u, the codec's is %lld", h.count, (long long)rk_rank(prm, d)); return FLC_ERR_ARG; }
            return FLC_OK;
        default:
            set_error("payload: unknown format %d", fmt);
            return FLC_ERR_UNSUPPORTED;
    }
}

size_t unpack_reduce_workspace(const flc_codec_params* prm, int64_t n, int64_t d) {
    if (payload_format(prm) == FMT_RANKK) return rk_unpack_workspace(prm, n, d);
    return payload_format(prm) == FMT_SPARSE ? sel_unpack_workspace(prm, n, d) : 0;
}

int unpack_reduce_run(const flc_codec_params* prm, const char* base, int64_t ld, const char* const* ptrs, int64_t n,
                      int64_t d, const float* w, float wt, float* out, void* ws, size_t ws_bytes, hipStream_t st) {
    if (d == 0) return FLC_OK;
    if (n == 0) { FLC_CHECK_HIP(hipMemsetAsync(out, 0, (size_t)d * sizeof(float), st)); return FLC_OK; }
    const int fmt = payload_format(prm);
    if (fmt == FMT_SPARSE) return sel_unpack_reduce(prm, base, ld, (const void* const*)ptrs, n, d, w, wt, out, ws, ws_bytes, st);
    if (fmt == FMT_RANKK) return rk_unpack_reduce(prm, base, ld, ptrs, n, d, w, wt, out, /*reduce=*/true, ws, ws_bytes, st);
    if (base && ((ld & 15) || ((uintptr_t)base & 15u))) { set_error("flc_unpack_reduce: payload rows must be 16-byte aligned"); return FLC_ERR_ARG; }
    const int E = fmt == FMT_Q8 ? 16 : (fmt == FMT_F32 ? 4 : 8);
    const int64_t groups = d / E + 1;
    const int grid = (int)((groups + 255) / 256);
    if (fmt == FMT_Q8 && prm->s > 127) { set_error("flc_unpack_reduce: Q8 with s > 127"); return FLC_ERR_ARG; }
#define UNPACK_CASE(F)                                                                                       \
    if (w) hipLaunchKernelGGL((k_unpack_accum<F, true, 4>), dim3(grid), dim3(256), 0, st, base, ld, ptrs, n, d,  \
                              prm->d_levels, prm->s, w, wt, out);                                            \
    else hipLaunchKernelGGL((k_unpack_accum<F, false, 4>), dim3(grid), dim3(256), 0, st, base, ld, ptrs, n, d,   \
                            prm->d_levels, prm->s, w, wt, out);
    { ProfScope _ps("k_unpack_accum", st);
    if (fmt == FMT_Q8) { UNPACK_CASE(FMT_Q8) }
    else if (fmt == FMT_Q16) { UNPACK_CASE(FMT_Q16) }
    else if (fmt == FMT_NAT16) { UNPACK_CASE(FMT_NAT16) }
    else { UNPACK_CASE(FMT_F32) } }
#undef UNPACK_CASE
    FLC_CHECK_LAUNCH("k_unpack_accum");
    return FLC_OK;
}

}  // namespace flc
