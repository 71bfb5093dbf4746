// Device/host helpers shared by the flcodec translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/flcodec.h"

namespace flc {

constexpr int WAVE = 64;          // CDNA wavefront
constexpr int CHUNK = 4096;       // elements per selection chunk (one wave's tile, 16 KB fp32)
constexpr int CHUNK_SHIFT = 12;

// ------------------------------------------------------------------------------------------
// error plumbing (thread-local message, status codes of flcodec.h)
// ------------------------------------------------------------------------------------------
void set_error(const char* fmt, ...);
int hip_fail(hipError_t e, const char* what);

#define FLC_CHECK_HIP(expr)                                          \
    do {                                                             \
        hipError_t _e = (expr);                                      \
        if (_e != hipSuccess) return ::flc::hip_fail(_e, #expr);     \
    } while (0)
#define FLC_CHECK_LAUNCH(what)                                       \
    do {                                                             \
        hipError_t _e = hipGetLastError();                           \
        if (_e != hipSuccess) return ::flc::hip_fail(_e, what);      \
    } while (0)

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Layout / probe switches for A/B tuning runs.  Only a build with -DFLC_TUNING (tools/ab_build.sh
// --tuning) reads them from the environment; the product library ignores the environment, so a
// stray variable can never change a result.
// Events that only order one device's streams (hipStreamWaitEvent; never inspected by the host):
// device-scope release, no system-scope cache writeback at each record
#ifndef FLC_SYNC_EVENT_FLAGS
#define FLC_SYNC_EVENT_FLAGS (hipEventDisableTiming | hipEventDisableSystemFence)
#endif

inline const char* tuning_env(const char* name) {
#ifdef FLC_TUNING
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

// Kernel timing (flc_profile_enable): a scope records a hipEvent pair around one launch.
extern bool g_prof_on;
void prof_record(const char* name, hipStream_t st, bool begin);
struct ProfScope {
    const char* name;
    hipStream_t st;
    ProfScope(const char* n, hipStream_t s) : name(n), st(s) { if (g_prof_on) prof_record(name, st, true); }
    ~ProfScope() { if (g_prof_on) prof_record(name, st, false); }
};

// Workspace carving: every sub-buffer 256-byte aligned.
struct Carver {
    char* base;
    size_t off = 0;
    explicit Carver(void* b) : base(static_cast<char*>(b)) {}
    template <class T>
    T* take(size_t count) {
        off = align_up(off, 256);
        T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
        off += count * sizeof(T);
        return p;
    }
    size_t bytes() const { return align_up(off, 256); }
};

// Row addressing shared by every kernel: a strided matrix (row i at base + i*ld) or a device
// array of row pointers (base == nullptr).
// Scalar (constant address space) load of a wave-uniform address: the data must not change
// during the kernel (written by earlier launches only).
template <class T>
__device__ inline T sload(const T* p) {
    return *(const __attribute__((address_space(4))) T*)p;
}

#ifndef FLC_ROWNT
#define FLC_ROWNT 1
#endif
// One float4 of a client row in a streaming pass (read once per launch): a nontemporal load
// (measured: the serverGradient fold 2-4 % faster, the dense norm pass 10 %; -DFLC_ROWNT=0 for A/B)
__device__ inline float4 ld_row4(const float4* p) {
#if FLC_ROWNT
    typedef float v4f __attribute__((ext_vector_type(4)));
    const v4f v = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
#else
    return *p;
#endif
}

struct RowSrc {
    const float* base;
    int64_t ld;
    const float* const* ptrs;
    __device__ inline const float* row(int64_t i) const { return base ? base + i * ld : ptrs[i]; }
    // wave-uniform i: the pointer table is read through the scalar cache (s_load, lgkmcnt), so it
    // does not join the vector-memory queue of a streaming pipeline
    __device__ inline const float* row_s(int64_t i) const {
        return base ? base + i * ld : sload(ptrs + i);
    }
};

// Internal entry points of the codec families (reduce.hip, codecs.hip, select.hip).
int reduce_impl(RowSrc src, bool rows_vec_ok, int64_t n, int64_t d, const float* x, const float* w, float wt,
                int mode, float* out, hipStream_t st);
size_t ew_workspace(const flc_codec_params* prm, int64_t n, int64_t d);
// The shift codecs' epilogue (flc_encode_shift): b is subtracted from the input row before the
// codec; msg = base + C * scale, hout = hin + alpha * C (null msg / hout: not written).
struct ShiftArgs {
    const float* b;
    float scale;
    const float* base;
    float* msg;
    float alpha;
    const float* hin;
    float* hout;
};
// flc_pack's fused encode -> code form (Q8 / Q16 / NAT16): payload header + body written directly
struct CodeArgs {
    int fmt;
    char* payload;
    const float* lv;     // the level table (dithering)
    int s;
    const float* pn;     // device norm the codes are relative to (dithering)
};
int ew_run(const flc_codec_params* prm, const flc_pattern* pat, RowSrc src, bool vec, int64_t n, int64_t d,
           const float* pnorm_in, float* pnorm_out, bool dense, float* out, const float* w, float wt, void* ws,
           size_t ws_bytes, hipStream_t st, const ShiftArgs* sh = nullptr, const CodeArgs* ca = nullptr);
size_t shift_workspace(const flc_codec_params* prm, int64_t d);
int encode_row(const flc_codec_params* prm, const flc_pattern* pat, const float* d_x, int64_t d,
               const float* d_pnorm_in, float* d_pnorm_out, float* d_out, void* d_ws, size_t ws_bytes, hipStream_t st);
size_t encode_row_workspace(const flc_codec_params* prm, int64_t d);
int sel_unpack_reduce(const flc_codec_params* prm, const void* base, int64_t ld_bytes, const void* const* ptrs,
                      int64_t n, int64_t d, const float* w, float wt, float* out, void* wsp, size_t ws_bytes,
                      hipStream_t st);
size_t sel_unpack_workspace(const flc_codec_params* prm, int64_t n, int64_t d);
int64_t payload_bytes(const flc_codec_params* prm, int64_t d);
int64_t rk_payload_floats(const flc_codec_params* prm, int64_t d);
int64_t rk_rank(const flc_codec_params* prm, int64_t d);
int rk_pack(const flc_codec_params* prm, const float* x, int64_t d, float* body, void* wsp, size_t ws_bytes,
            hipStream_t st);
size_t rk_unpack_workspace(const flc_codec_params* prm, int64_t n, int64_t d);
int rk_unpack1(const flc_codec_params* prm, const float* body, int64_t d, float* out, hipStream_t st);
int rk_unpack_reduce(const flc_codec_params* prm, const char* base, int64_t ld, const char* const* ptrs, int64_t n,
                     int64_t d, const float* w, float wt, float* out, bool reduce, void* wsp, size_t ws_bytes,
                     hipStream_t st);
int payload_format(const flc_codec_params* prm);
int payload_validate(const flc_codec_params* prm, const uint8_t* p, int64_t nbytes, int64_t d);
size_t pack_workspace(const flc_codec_params* prm, int64_t d);
int pack_run(const flc_codec_params* prm, const flc_pattern* pat, const float* x, int64_t d, char* payload, void* ws,
             size_t ws_bytes, hipStream_t st);
int unpack_run(const flc_codec_params* prm, const char* payload, int64_t d, float* out, hipStream_t st);
size_t unpack_reduce_workspace(const flc_codec_params* prm, int64_t n, int64_t d);
int unpack_reduce_run(const flc_codec_params* prm, const char* base, int64_t ld, const char* const* ptrs, int64_t n,
                      int64_t d, const float* w, float wt, float* out, void* ws, size_t ws_bytes, hipStream_t st);
int shift_run(const flc_codec_params* prm, const flc_pattern* pat, const float* a, int64_t d, const ShiftArgs& sh,
              float* pnorm_out, void* ws, size_t ws_bytes, hipStream_t st);
// Row g's boundary of G row groups whose last group is `lastpct` % of the others' size (the last
// group's tail is the exposed one): rows [group_row(n, G, g), group_row(n, G, g + 1)).
// lastpct is clamped to [1, 100]: 0 or less would leave the last group (the one whose fold writes
// the output) empty, above 100 is the even split.
inline int64_t group_row(int64_t n, int G, int g, int lastpct) {
    lastpct = lastpct < 1 ? 1 : lastpct;
    if (G <= 1 || lastpct >= 100) return n * g / G;
    const int64_t unit = 100 * (int64_t)(G - 1) + lastpct;     // group sizes 100, ..., 100, lastpct
    const int64_t cum = g <= G - 1 ? 100 * (int64_t)g : unit;
    return n * cum / unit;
}
int norm_torch_run(const float* x, int64_t ld, int64_t n, int64_t d, float* out, hipStream_t st);
size_t norm_torch_ws_bytes(int64_t n, int64_t d);
int norm_torch_ws_run(const float* x, int64_t ld, int64_t n, int64_t d, float* out, void* wsp, size_t ws_bytes,
                      hipStream_t st);
size_t sel_workspace(const flc_codec_params* prm, int64_t n, int64_t d);
int sel_run(const flc_codec_params* prm, const flc_pattern* pat, RowSrc rows, bool vec, int64_t n, int64_t d,
            bool assign, const float* w, float wt, float* out, void* wsp, size_t ws_bytes, hipStream_t st);
int rs_debug(int mult, int64_t spin_ticks);
int sel_row_flags(const flc_codec_params* prm, int64_t n, int64_t d, const void* wsp, size_t ws_bytes,
                  uint32_t* flags, hipStream_t st);
bool ds_eligible(const flc_codec_params* prm, const flc_pattern* pat, int64_t n, int64_t d);
size_t ds_workspace(const flc_codec_params* prm, int64_t n, int64_t d);
int ds_run(const flc_codec_params* prm, const flc_pattern* pat, RowSrc rows, int64_t n, int64_t d, const float* w,
           float wt, float* pnorm_out, float* out, void* wsp, size_t ws_bytes, hipStream_t st);
size_t rk_workspace(const flc_codec_params* prm, int64_t n, int64_t d, bool reduce);
int rk_run(const flc_codec_params* prm, RowSrc rows, int64_t n, int64_t d, bool reduce, const float* w, float wt,
           float* out, void* wsp, size_t ws_bytes, hipStream_t st);
size_t randk_device_workspace(int64_t n, int64_t d);
int randk_device_counts(uint64_t seed, int64_t client0, int64_t n, int64_t d, int64_t k, uint32_t* cnt, void* ws,
                        size_t ws_bytes, hipStream_t st);
int randk_dense(const flc_codec_params* prm, const flc_pattern* pat, const float* x, int64_t d, float* out, void* ws,
                size_t ws_bytes,
                hipStream_t st);

// ------------------------------------------------------------------------------------------
// Device-RNG mode: counter-based generator, SplitMix64 finaliser over a keyed Weyl sequence.
// uniform(seed, client, j) = (mix(seed, client, j) >> 11) * 2^-53 — a 53-bit double like
// numpy's random_sample, so compat and device modes share every downstream comparison.
// ------------------------------------------------------------------------------------------
__host__ __device__ inline uint64_t mix64(uint64_t z) {
    z ^= z >> 30;
    z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27;
    z *= 0x94D049BB133111EBull;
    z ^= z >> 31;
    return z;
}
__host__ __device__ inline uint64_t client_key(uint64_t seed, int64_t client) {
    return mix64(seed ^ mix64(0x9E3779B97F4A7C15ull * (uint64_t)(client + 1)));
}
__host__ __device__ inline double uniform53(uint64_t ckey, int64_t j) {
    uint64_t z = mix64(ckey + 0x9E3779B97F4A7C15ull * (uint64_t)j);
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

// Per-element device draw used by the dithering / natural kernels: a 32-bit uniform
// u = fmix32(j * m_c + o_c) * 2^-32, with (m_c odd, o_c) taken from the client key — one Weyl
// sequence per client through the MurmurHash3 finaliser (a bijection with full avalanche).
// 32-bit multiplies only: the 64-bit mix above costs ~3x the VALU time per element.
__host__ __device__ inline uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}
// u(client, j) = hi8 << 24 | lo24 from two hashes keyed by the row key rk (a 32-bit fold of the
// client key):
//   lo24 = fmix32(colbase(j) + (rk ^ 0x27D4EB2F)) >> 8,  colbase(j) = j * 0x85EBCA77 (computed
//          once per column by the tile-owner kernels, outside the client loop);
//   hi8  = byte (j & 3) of grouphash(j >> 2, rk) = gmix((j >> 2) * 0x9E3779B1 + rk) — one hash
//          serves 4 consecutive elements.
// The split lets a streaming pass decide `u >= t` for a small t from the top byte alone, at a
// quarter hash per element (the sparse QSGD candidate filter, dither_sparse.hip).  gmix is two
// rounds of xorshift + 24-bit multiply (v_mul_u32_u24, full rate; the top byte the multiply ignores
// is xored back in), instead of the MurmurHash3 finaliser's two quarter-rate 32-bit multiplies:
// same-box A/B 0.1-0.2 ms off the C4 filter; statistically checked like fmix32 (bit bias, bit-pair
// correlations at lags 0-1024, 4-byte joint, adjacent groups: tests/test_host.py).
__host__ __device__ inline uint32_t colbase(uint32_t j) { return j * 0x85EBCA77u; }
__host__ __device__ inline uint32_t rowkey(uint64_t ckey) { return (uint32_t)(ckey >> 32) ^ (uint32_t)ckey; }
#ifndef FLC_GHASH
#define FLC_GHASH 1
#endif
__host__ __device__ inline uint32_t mul24(uint32_t a, uint32_t b) { return (a & 0xFFFFFFu) * (b & 0xFFFFFFu); }
// FLC_GHASH (A/B builds only; the draws are part of the device-RNG definition and oracle/devrng.py
// states variant 1): 0 = fmix32, 1 = the 24-bit mixer, 2 = a 32x32->64 multiply folded lo ^ hi
__host__ __device__ inline uint32_t gmix(uint32_t v) {
#if FLC_GHASH == 1
    uint32_t h = v ^ (v >> 16);
    h = mul24(h, 0xB5297Bu) ^ (h >> 24);
    h ^= h >> 16;
    h = mul24(h, 0x68E31Du) ^ (h >> 24);
    return h ^ (h >> 16);
#elif FLC_GHASH == 2
    const uint64_t p = (uint64_t)v * (uint64_t)(v ^ 0x2D358DCCu);
    return (uint32_t)p ^ (uint32_t)(p >> 32);
#else
    return fmix32(v);
#endif
}
__host__ __device__ inline uint32_t grouphash(uint32_t g, uint32_t rk) { return gmix(g * 0x9E3779B1u + rk); }
__host__ __device__ inline uint32_t draw_join(uint32_t hg, uint32_t q, uint32_t lo) {
    return ((hg >> (8u * q)) << 24) | (lo >> 8);
}
__host__ __device__ inline uint32_t dev_draw(uint32_t cs, uint32_t hg, uint32_t j, uint32_t rk) {
    return draw_join(hg, j & 3u, fmix32(cs + (rk ^ 0x27D4EB2Fu)));
}
__host__ __device__ inline uint32_t dev_u32(uint64_t ckey, uint32_t j) {
    const uint32_t rk = rowkey(ckey);
    return dev_draw(colbase(j), grouphash(j >> 2, rk), j, rk);
}
// Decision for a draw h (u = h * 2^-32) against an fp32 probability p:  h < sat_u32(ceil(p*2^32)).
// Equals (u < p) exactly for p in [0, 1); p >= 1 admits every h but 0xFFFFFFFF (prob. 2^-32), and
// p <= 0 or NaN admits none.  ldexp / ceil / saturating convert are exact single instructions.
__host__ __device__ inline uint32_t thr32(float p) {
    const float t = ceilf(ldexpf(p, 32));
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;   // v_cvt_u32_f32 saturates: < 0 -> 0, >= 2^32 -> 0xFFFFFFFF, NaN -> 0
    asm("v_cvt_u32_f32 %0, %1" : "=v"(r) : "v"(t));
    return r;
#else
    if (!(t > 0.f)) return 0u;                    // p <= 0 or NaN
    if (t >= 4294967295.f) return 0xFFFFFFFFu;
    return (uint32_t)t;
#endif
}
__host__ __device__ inline bool below32(uint32_t h, float p) { return h < thr32(p); }

// ------------------------------------------------------------------------------------------
// Wave helpers
// ------------------------------------------------------------------------------------------
__device__ inline int lane_id() { return __lane_id(); }

template <class T>
__device__ inline T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
    return v;
}

// |x| ordering key for TopK: sign cleared; NaN (0x7F8..1-0x7FF..F) above +inf, like torch.topk.
__device__ inline uint32_t mag_key(float x) { return __float_as_uint(x) & 0x7FFFFFFFu; }

// torch.sign semantics: -1 / 0 / +1 (NaN -> 0 is irrelevant: a NaN row's norm is NaN).
__device__ inline float tsign(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

}  // namespace flc
