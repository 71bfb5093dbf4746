// C ABI entry points of libflcodec.so (declared in include/flcodec.h): argument checking,
// workspace sizing and dispatch to the codec families.
#include <stdarg.h>
#include <stdio.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "common.hpp"

namespace flc {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int hip_fail(hipError_t e, const char* what) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return FLC_ERR_HIP;
}

// ---- kernel timing ------------------------------------------------------------------------
bool g_prof_on = false;
namespace {
std::mutex g_prof_mu;
std::vector<hipEvent_t> g_ev_free;
std::map<std::string, std::vector<std::pair<hipEvent_t, hipEvent_t>>> g_prof;
std::map<std::string, hipEvent_t> g_open;
hipEvent_t take_event() {
    if (!g_ev_free.empty()) { hipEvent_t e = g_ev_free.back(); g_ev_free.pop_back(); return e; }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}
}  // namespace

void prof_record(const char* name, hipStream_t st, bool begin) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    hipEvent_t e = take_event();
    if (!e) return;
    (void)hipEventRecord(e, st);
    if (begin) {
        g_open[name] = e;
    } else {
        auto it = g_open.find(name);
        if (it == g_open.end()) { g_ev_free.push_back(e); return; }
        g_prof[name].emplace_back(it->second, e);
        g_open.erase(it);
    }
}

static bool is_sel(int codec) { return codec == FLC_TOPK || codec == FLC_RANDK; }
static bool known(int codec) { return codec >= FLC_IDENT && codec <= FLC_RANK_K; }
// host-side check of the fields that choose WHAT is computed (before any device argument)
static int bad_params(const flc_codec_params* prm, const char* what) {
    if (prm->codec == FLC_TOPK && prm->tie != FLC_TIE_LOWEST && prm->tie != FLC_TIE_HIGHEST) {
        set_error("%s: unknown TopK tie rule %d (FLC_TIE_LOWEST / FLC_TIE_HIGHEST)", what, (int)prm->tie);
        return FLC_ERR_ARG;
    }
    return FLC_OK;
}

}  // namespace flc

using namespace flc;

extern "C" int flc_version(void) { return 104; }   // 1.04: flc_rows_alloc / free (1.03: flc_norm2_torch_cpu_ws; 1.02: flc_debug_resident; 1.01: tie, flc_norm2_torch_cpu)

#ifndef FLC_SRC_HASH
#define FLC_SRC_HASH "unknown"
#endif
extern "C" const char* flc_build_id(void) { return FLC_SRC_HASH; }

extern "C" int flc_profile_enable(int on) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof_on = on != 0;
    return FLC_OK;
}

extern "C" int flc_profile_collect(const char* kernel, double* h_total_ms, int64_t* h_launches) {
    if (!kernel || !h_total_ms || !h_launches) { set_error("flc_profile_collect: null argument"); return FLC_ERR_ARG; }
    std::vector<std::pair<hipEvent_t, hipEvent_t>> recs;
    {
        std::lock_guard<std::mutex> lk(g_prof_mu);
        auto it = g_prof.find(kernel);
        if (it != g_prof.end()) { recs.swap(it->second); g_prof.erase(it); }
    }
    double total = 0.0;
    for (auto& r : recs) {
        FLC_CHECK_HIP(hipEventSynchronize(r.second));
        float ms = 0.f;
        FLC_CHECK_HIP(hipEventElapsedTime(&ms, r.first, r.second));
        total += ms;
    }
    {
        std::lock_guard<std::mutex> lk(g_prof_mu);
        for (auto& r : recs) { g_ev_free.push_back(r.first); g_ev_free.push_back(r.second); }
    }
    *h_total_ms = total;
    *h_launches = (int64_t)recs.size();
    return FLC_OK;
}

extern "C" const char* flc_last_error_string(void) { return g_err; }

extern "C" int flc_select_row_flags(const flc_codec_params* prm, int64_t n, int64_t d, const void* d_workspace,
                                    size_t ws_bytes, uint32_t* d_flags, void* stream) {
    if (!prm || (n > 0 && (!d_workspace || !d_flags))) { set_error("flc_select_row_flags: null argument"); return FLC_ERR_ARG; }
    return sel_row_flags(prm, n, d, d_workspace, ws_bytes, d_flags, (hipStream_t)stream);
}

// Host helper (no compute): the resident client-update matrix in PHYSICALLY CONTIGUOUS HBM
// (hipDeviceMallocContiguous).  A default allocation of tens of GB is stitched from fragments and
// some of its rows read 6-10 % slower, with more address-translation misses (profiles/r06/
// regions_pmc.jsonl); contiguous memory maps with the largest page fragments: C4's 51.2 GB shard
// read 8.04 vs 8.48 ms, its step 9.09 vs 9.57 ms, same process (profiles/r06/contig.jsonl).
extern "C" int flc_rows_alloc(size_t bytes, int contiguous, void** d_ptr) {
    if (!d_ptr || bytes == 0) { set_error("flc_rows_alloc: bad args"); return FLC_ERR_ARG; }
    *d_ptr = nullptr;
    const hipError_t e = contiguous ? hipExtMallocWithFlags(d_ptr, bytes, hipDeviceMallocContiguous) : hipMalloc(d_ptr, bytes);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        *d_ptr = nullptr;
        set_error("flc_rows_alloc: %s of %zu bytes failed: %s", contiguous ? "contiguous allocation" : "hipMalloc", bytes,
                  hipGetErrorString(e));
        return FLC_ERR_HIP;
    }
    return FLC_OK;
}

extern "C" int flc_rows_free(void* d_ptr) {
    if (d_ptr && hipFree(d_ptr) != hipSuccess) { set_error("flc_rows_free: hipFree failed"); return FLC_ERR_HIP; }
    return FLC_OK;
}

extern "C" size_t flc_norm2_torch_cpu_workspace_size(int64_t n, int64_t d) {
    return (n <= 0 || d < 0) ? 0 : norm_torch_ws_bytes(n, d);
}

extern "C" int flc_norm2_torch_cpu_ws(const float* d_rows, int64_t ld, int64_t n, int64_t d, float* d_out, void* d_ws,
                                      size_t ws_bytes, void* stream) {
    if (n < 0 || d < 0 || (n > 1 && ld < d) || (n > 0 && (!d_rows || !d_out || !d_ws))) {
        set_error("flc_norm2_torch_cpu_ws: bad args (n=%lld d=%lld ld=%lld)", (long long)n, (long long)d, (long long)ld);
        return FLC_ERR_ARG;
    }
    if (n == 0) return FLC_OK;
    return norm_torch_ws_run(d_rows, ld, n, d, d_out, d_ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int flc_debug_resident(int grid_mult, int64_t spin_ticks) { return rs_debug(grid_mult, spin_ticks); }

extern "C" int flc_norm2_torch_cpu(const float* d_rows, int64_t ld, int64_t n, int64_t d, float* d_out, void* stream) {
    if (n < 0 || d < 0 || (n > 1 && ld < d) || (n > 0 && (!d_rows || !d_out))) {
        set_error("flc_norm2_torch_cpu: bad args (n=%lld d=%lld ld=%lld)", (long long)n, (long long)d, (long long)ld);
        return FLC_ERR_ARG;
    }
    if (n == 0) return FLC_OK;
    return norm_torch_run(d_rows, ld, n, d, d_out, (hipStream_t)stream);
}

namespace flc {
int selftest_division(const float* d_b, int nb, unsigned long long* d_bad, hipStream_t st);
}
extern "C" int flc_selftest_division(const float* d_divisors, int n, unsigned long long* d_mismatches,
                                     void* stream) {
    if (n < 0 || (n > 0 && (!d_divisors || !d_mismatches))) { set_error("flc_selftest_division: bad args"); return FLC_ERR_ARG; }
    if (n == 0) return FLC_OK;
    return selftest_division(d_divisors, n, d_mismatches, (hipStream_t)stream);
}

namespace flc {
size_t encode_row_workspace(const flc_codec_params* prm, int64_t d) {
    if (prm->codec == FLC_TOPK) return sel_workspace(prm, 1, d);
    if (prm->codec == FLC_RANK_K) return rk_workspace(prm, 1, d, false);
    if (prm->codec == FLC_RANDK) return randk_device_workspace(1, d);
    return ew_workspace(prm, 1, d);
}
}  // namespace flc

extern "C" size_t flc_encode_workspace_size(const flc_codec_params* prm, int64_t d) {
    if (!prm || !known(prm->codec)) return 0;
    if (prm->codec == FLC_TOPK) return sel_workspace(prm, 1, d);
    if (prm->codec == FLC_RANK_K) return rk_workspace(prm, 1, d, false);
    if (prm->codec == FLC_RANDK) return randk_device_workspace(1, d);
    return ew_workspace(prm, 1, d);
}

extern "C" size_t flc_encode_reduce_workspace_size(const flc_codec_params* prm, int64_t n, int64_t d) {
    if (!prm || !known(prm->codec)) return 0;
    if (is_sel(prm->codec)) return sel_workspace(prm, n, d);
    if (prm->codec == FLC_RANK_K) return rk_workspace(prm, n, d, true);
    return ew_workspace(prm, n, d);
}

namespace flc {
// one row, dense output (flc_encode; also the first stage of flc_pack)
int encode_row(const flc_codec_params* prm, const flc_pattern* pat, const float* d_x, int64_t d,
               const float* d_pnorm_in, float* d_pnorm_out, float* d_out, void* d_ws, size_t ws_bytes, hipStream_t st) {
    const bool vec = (((uintptr_t)d_x | (uintptr_t)d_out) & 15u) == 0;
    switch (prm->codec) {
        case FLC_RANDK:
            if (!(pat && pat->d_randk_idx) && prm->k > d) { set_error("randk: K > D"); return FLC_ERR_ARG; }
            return randk_dense(prm, pat, d_x, d, d_out, d_ws, ws_bytes, st);
        case FLC_RANK_K: {
            RowSrc r{d_x, d, nullptr};
            return rk_run(prm, r, 1, d, /*reduce=*/false, nullptr, 1.f, d_out, d_ws, ws_bytes, st);
        }
        case FLC_TOPK: {
            RowSrc r{d_x, d, nullptr};
            return sel_run(prm, pat, r, vec, 1, d, /*assign=*/true, nullptr, 1.f, d_out, d_ws, ws_bytes, st);
        }
        default: {
            RowSrc s{d_x, d, nullptr};
            return ew_run(prm, pat, s, vec, 1, d, d_pnorm_in, d_pnorm_out, /*dense=*/true, d_out, nullptr, 1.f, d_ws,
                          ws_bytes, st);
        }
    }
}
}  // namespace flc

extern "C" int flc_encode(const flc_codec_params* prm, const flc_pattern* pat, const float* d_x, int64_t d,
                          const float* d_pnorm_in, float* d_pnorm_out, float* d_out, void* d_ws, size_t ws_bytes,
                          void* stream) {
    if (!prm || !known(prm->codec)) { set_error("flc_encode: unknown codec"); return FLC_ERR_UNSUPPORTED; }
    if (int rc = bad_params(prm, "flc_encode")) return rc;
    if (d < 0 || (d > 0 && (!d_x || !d_out))) { set_error("flc_encode: bad x/out/d"); return FLC_ERR_ARG; }
    return encode_row(prm, pat, d_x, d, d_pnorm_in, d_pnorm_out, d_out, d_ws, ws_bytes, (hipStream_t)stream);
}

extern "C" size_t flc_encode_shift_workspace_size(const flc_codec_params* prm, int64_t d) {
    if (!prm || !known(prm->codec) || d < 0) return 0;
    return shift_workspace(prm, d);
}

extern "C" int flc_encode_shift(const flc_codec_params* prm, const flc_pattern* pat, const float* d_a,
                                const float* d_b, int64_t d, float msg_scale, const float* d_base, float* d_msg,
                                float shift_alpha, const float* d_shift_in, float* d_shift_out, float* d_pnorm_out,
                                void* d_ws, size_t ws_bytes, void* stream) {
    if (!prm || !known(prm->codec)) { set_error("flc_encode_shift: unknown codec"); return FLC_ERR_UNSUPPORTED; }
    if (int rc = bad_params(prm, "flc_encode_shift")) return rc;
    if (d < 0) { set_error("flc_encode_shift: d < 0"); return FLC_ERR_ARG; }
    if (d > 0 && (!d_a || !d_b)) { set_error("flc_encode_shift: need a and b"); return FLC_ERR_ARG; }
    if (d > 0 && !d_msg && !d_shift_out) { set_error("flc_encode_shift: nothing to write (msg and shift_out null)"); return FLC_ERR_ARG; }
    if (d_shift_out && !d_shift_in) { set_error("flc_encode_shift: shift_out without shift_in"); return FLC_ERR_ARG; }
    if (d_base && !d_msg) { set_error("flc_encode_shift: base without msg"); return FLC_ERR_ARG; }
    ShiftArgs sh{d_b, msg_scale, d_base, d_msg, shift_alpha, d_shift_in, d_shift_out};
    return shift_run(prm, pat, d_a, d, sh, d_pnorm_out, d_ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int64_t flc_payload_bytes(const flc_codec_params* prm, int64_t d) {
    if (!prm || !known(prm->codec) || d < 0) return 0;
    return payload_bytes(prm, d);
}

extern "C" int flc_payload_format(const flc_codec_params* prm) {
    if (!prm || !known(prm->codec)) return 0;
    return payload_format(prm);
}

extern "C" int flc_payload_validate(const flc_codec_params* prm, const void* h_payload, int64_t nbytes, int64_t d) {
    if (!prm || !known(prm->codec)) { set_error("flc_payload_validate: unknown codec"); return FLC_ERR_UNSUPPORTED; }
    if (d < 0 || nbytes < 0 || (nbytes > 0 && !h_payload)) { set_error("flc_payload_validate: bad payload/nbytes/d"); return FLC_ERR_ARG; }
    return payload_validate(prm, (const uint8_t*)h_payload, nbytes, d);
}

extern "C" size_t flc_pack_workspace_size(const flc_codec_params* prm, int64_t d) {
    if (!prm || !known(prm->codec) || d < 0) return 0;
    return pack_workspace(prm, d);
}

extern "C" int flc_pack(const flc_codec_params* prm, const flc_pattern* pat, const float* d_x, int64_t d,
                        void* d_payload, void* d_ws, size_t ws_bytes, void* stream) {
    if (!prm || !known(prm->codec)) { set_error("flc_pack: unknown codec"); return FLC_ERR_UNSUPPORTED; }
    if (int rc = bad_params(prm, "flc_pack")) return rc;
    if (d < 0 || !d_payload || (d > 0 && !d_x)) { set_error("flc_pack: bad x/payload/d"); return FLC_ERR_ARG; }
    return pack_run(prm, pat, d_x, d, (char*)d_payload, d_ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int flc_unpack(const flc_codec_params* prm, const void* d_payload, int64_t d, float* d_out, void* stream) {
    if (!prm || !known(prm->codec)) { set_error("flc_unpack: unknown codec"); return FLC_ERR_UNSUPPORTED; }
    if (d < 0 || (d > 0 && (!d_payload || !d_out))) { set_error("flc_unpack: bad payload/out/d"); return FLC_ERR_ARG; }
    return unpack_run(prm, (const char*)d_payload, d, d_out, (hipStream_t)stream);
}

extern "C" size_t flc_unpack_reduce_workspace_size(const flc_codec_params* prm, int64_t n, int64_t d) {
    if (!prm || !known(prm->codec) || n < 0 || d < 0) return 0;
    return unpack_reduce_workspace(prm, n, d);
}

extern "C" int flc_unpack_reduce(const flc_codec_params* prm, const void* d_payloads, int64_t ld_bytes,
                                 const void* const* d_payload_ptrs, int64_t n, int64_t d, const float* d_w,
                                 float w_total, float* d_out, void* d_ws, size_t ws_bytes, void* stream) {
    if (!prm || !known(prm->codec)) { set_error("flc_unpack_reduce: unknown codec"); return FLC_ERR_UNSUPPORTED; }
    if (n < 0 || d < 0 || (d > 0 && !d_out)) { set_error("flc_unpack_reduce: bad n/d/out"); return FLC_ERR_ARG; }
    if (n > FLC_MAX_ROWS) {
        set_error("flc_unpack_reduce: n=%lld payloads, at most %d per call", (long long)n, FLC_MAX_ROWS);
        return FLC_ERR_UNSUPPORTED;
    }
    if (n > 0 && d > 0 && !d_payloads && !d_payload_ptrs) { set_error("flc_unpack_reduce: no payloads"); return FLC_ERR_ARG; }
    if (d_payloads && ld_bytes < payload_bytes(prm, d)) { set_error("flc_unpack_reduce: ld_bytes < payload size"); return FLC_ERR_ARG; }
    return unpack_reduce_run(prm, (const char*)d_payloads, ld_bytes, (const char* const*)d_payload_ptrs, n, d, d_w,
                             w_total, d_out, d_ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int flc_encode_reduce(const flc_codec_params* prm, const flc_pattern* pat, const float* d_rows, int64_t ld,
                                 const float* const* d_row_ptrs, int64_t n, int64_t d, const float* d_w, float w_total,
                                 float* d_pnorms_out, float* d_out, void* d_ws, size_t ws_bytes, void* stream) {
    if (!prm || !known(prm->codec)) { set_error("flc_encode_reduce: unknown codec"); return FLC_ERR_UNSUPPORTED; }
    if (int rc = bad_params(prm, "flc_encode_reduce")) return rc;
    if (n < 0 || d < 0 || (d > 0 && !d_out)) { set_error("flc_encode_reduce: bad n/d/out"); return FLC_ERR_ARG; }
    if (n > FLC_MAX_ROWS) {   // per-row kernels index rows by blockIdx.y
        set_error("flc_encode_reduce: n=%lld rows, at most %d per call (fold larger rounds as partials)", (long long)n,
                  FLC_MAX_ROWS);
        return FLC_ERR_UNSUPPORTED;
    }
    if (n > 0 && d > 0 && !d_rows && !d_row_ptrs) { set_error("flc_encode_reduce: no rows"); return FLC_ERR_ARG; }
    if (d_rows && ld < d) { set_error("flc_encode_reduce: ld < d"); return FLC_ERR_ARG; }
    hipStream_t st = (hipStream_t)stream;
    if (d == 0) return FLC_OK;
    if (n == 0) {
        FLC_CHECK_HIP(hipMemsetAsync(d_out, 0, (size_t)d * sizeof(float), st));
        return FLC_OK;
    }
    // vector path: matrix rows 16-byte aligned with ld % 4 == 0; pointer rows are required aligned
    const bool vec = d_rows ? ((((uintptr_t)d_rows & 15u) == 0) && (ld % 4 == 0)) : true;
    if (prm->codec == FLC_IDENT) {
        RowSrc s{d_rows, ld, d_row_ptrs};
        return reduce_impl(s, vec, n, d, nullptr, d_w, w_total, FLC_REDUCE_PLAIN, d_out, st);
    }
    if (prm->codec == FLC_RANK_K) {
        RowSrc r{d_rows, ld, d_row_ptrs};
        return rk_run(prm, r, n, d, /*reduce=*/true, d_w, w_total, d_out, d_ws, ws_bytes, st);
    }
    if (is_sel(prm->codec)) {
        RowSrc r{d_rows, ld, d_row_ptrs};
        return sel_run(prm, pat, r, vec, n, d, false, d_w, w_total, d_out, d_ws, ws_bytes, st);
    }
    RowSrc s{d_rows, ld, d_row_ptrs};
    return ew_run(prm, pat, s, vec, n, d, nullptr, d_pnorms_out, false, d_out, d_w, w_total, d_ws, ws_bytes, st);
}

extern "C" size_t flc_device_randk_counts_workspace_size(int64_t n, int64_t d) {
    if (n < 1 || d < 1) return 0;
    return randk_device_workspace(n, d);
}

extern "C" int flc_device_randk_counts(uint64_t seed, int64_t client0, int64_t n, int64_t d, int64_t k,
                                       uint32_t* d_counts, void* d_ws, size_t ws_bytes, void* stream) {
    if (n < 1 || d < 1 || k < 1 || k > d || d >= (int64_t)0xFFFFFFFF || !d_counts) {
        set_error("flc_device_randk_counts: bad arguments");
        return FLC_ERR_ARG;
    }
    if (n > FLC_MAX_ROWS) {   // k_randk_counts indexes rows by blockIdx.y
        set_error("flc_device_randk_counts: n=%lld rows, at most %d per call", (long long)n, FLC_MAX_ROWS);
        return FLC_ERR_UNSUPPORTED;
    }
    return randk_device_counts(seed, client0, n, d, k, d_counts, d_ws, ws_bytes, (hipStream_t)stream);
}
