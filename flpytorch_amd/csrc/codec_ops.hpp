// Per-element codec functors shared by the dense / tile-owner kernels (codecs.hip) and the sparse
// dithering path (dither_sparse.hip): exact fp32 division, the device-RNG decision, and the
// ident / lazy / natural / standard-dithering element maps of fl_pytorch/utils/compressors.py.
#pragma once
#include "common.hpp"

namespace flc {

// ------------------------------------------------------------------------------------------
// Exact fp32 division, fast.  For a fixed divisor b with rb = RN(1/b) (IEEE, once per row or
// per level interval), Markstein's sequence  q0 = a*rb; r = fma(-q0, b, a) (exact);
// q = fma(r, rb, q0)  is the correctly rounded a/b when nothing under/overflows (Markstein
// 1990; Muller et al., Handbook of FP Arithmetic, "Markstein's theorem").  a/b of two floats is
// never a rounding midpoint, so the tiny error of rb cannot flip a tie.  The window: divisor in
// [2^-40, 2^80], numerator 0 or in [2^-80, 2^80] (below, r or q underflows and the identity
// fails — measured); elsewhere the IEEE division.  The norm pass marks rows whose every element
// is inside the window (rowfast), so their |x|/pnorm takes div_fast with no per-element guard.
// tests/test_gpu_parity.py checks the identity exhaustively, for a set of divisors, over EVERY
// float numerator of the window (flc_selftest_division).
// ------------------------------------------------------------------------------------------
struct FastDiv {
    float b, rb;
    bool ok;
};
__device__ inline FastDiv make_div(float b) {
    FastDiv f;
    f.b = b;
    f.rb = 1.0f / b;
    const float ab = fabsf(b);
    f.ok = ab >= 0x1p-40f && ab <= 0x1p80f;   // also false for NaN
    return f;
}
__device__ inline float div_fast(float a, const FastDiv& f) {   // caller guarantees the window
    const float q0 = a * f.rb;
    const float r = fmaf(-q0, f.b, a);
    return fmaf(r, f.rb, q0);
}
__device__ inline float div_rn(float a, const FastDiv& f) {
    const float aa = fabsf(a);
    if (f.ok && (aa == 0.f || (aa >= 0x1p-80f && aa <= 0x1p80f))) return div_fast(a, f);
    return a / f.b;
}

// ------------------------------------------------------------------------------------------
// Per-row state, computed once per row (k_norm_final / k_row_keys), read by the element loops
// with scalar loads: the norm, its reciprocal (div_fast), the fast-window flag and the device
// RNG row key.  Per-column state (the hashed element index) is computed once per column.
// ------------------------------------------------------------------------------------------
struct RowTabs {
    const float* pn;        // [n] norm
    const float* rpn;       // [n] RN(1/norm)
    const uint32_t* fast;   // [n] row inside the div_fast window (nullptr: guarded path)
    const uint32_t* rk;     // [n] device-RNG row key (nullptr in compat mode)
};

struct UniformSrc {
    const double* u;        // compat: [n][uld] float64 numpy draws
    int64_t uld;
};

// the reference's decision `testp < p` (float64 draw vs fp32 p promoted), compressors.py:260, 288.
// Device mode: h = dev_draw(colbase(j), grouphash, j, rowkey) against thr32 (common.hpp); p2 = p * 2^32.
// hg: grouphash(j >> 2, rk), shared by the 4 elements of an aligned group (hg_of below for one
// element).
template <bool COMPAT>
__device__ inline bool draw_below(const double* urow, uint32_t rk, int64_t j, uint32_t cs, uint32_t hg, float p,
                                  float p2) {
    if (COMPAT) return urow[j] < (double)p;
    uint32_t t;
    asm("v_cvt_u32_f32 %0, %1" : "=v"(t) : "v"(ceilf(p2)));   // saturating: thr32(p)
    // the draw's top byte decides unless it equals t's (1 in 256): only those lanes hash the low part
    const uint32_t hi8 = (hg >> (8u * ((uint32_t)j & 3u))) & 0xFFu, th = t >> 24;
    bool below = hi8 < th;
    const bool tie = hi8 == th;
    if (__builtin_expect(__ballot(tie) != 0ull, 0)) {
        if (tie) below = dev_draw(cs, hg, (uint32_t)j, rk) < t;
    }
    return below;
}
template <bool COMPAT>
__device__ inline uint32_t hg_of(uint32_t rk, int64_t j) { return COMPAT ? 0u : grouphash((uint32_t)(j >> 2), rk); }

// ------------------------------------------------------------------------------------------
// Per-element codecs.  setup(row) loads row-uniform state; col(j) is the per-column state
// (hoisted out of the row loop); apply<F>(x, j, cs, tab) -> C(x)[j].  `tab` is the LDS level
// table passed straight from the kernel's __shared__ array.
// ------------------------------------------------------------------------------------------
struct IdentOp {
    static constexpr bool TABLE = false;
    static constexpr bool HAS_APPLY4 = false;
    __device__ inline void setup(int64_t) {}
    __device__ inline bool row_fast() const { return false; }
    __device__ inline void set_table_ok(bool) {}
    __device__ inline uint32_t col(int64_t) const { return 0u; }
    template <bool F>
    __device__ inline float apply(float x, int64_t, uint32_t, const float4*) const { return x; }
};

struct LazyOp {                       // compressors.py:231-238: x / P if testp < P else 0
    static constexpr bool TABLE = false;
    static constexpr bool HAS_APPLY4 = false;
    const double* lazy_u;             // [n] float64 draws (numpy random())
    float P;
    bool keep;
    __device__ inline void setup(int64_t row) { keep = lazy_u[row] < (double)P; }
    __device__ inline bool row_fast() const { return false; }
    __device__ inline void set_table_ok(bool) {}
    __device__ inline uint32_t col(int64_t) const { return 0u; }
    template <bool F>
    __device__ inline float apply(float x, int64_t, uint32_t, const float4*) const { return keep ? x / P : 0.f; }
};

template <bool COMPAT>
struct NaturalOp {                    // compressors.py:247-268
    static constexpr bool TABLE = false;
    static constexpr bool HAS_APPLY4 = false;
    UniformSrc us;
    const uint32_t* rks;
    const double* urow;
    uint32_t rk;
    __device__ inline void setup(int64_t row) {
        urow = COMPAT ? us.u + row * us.uld : nullptr;
        rk = COMPAT ? 0u : rks[row];
    }
    __device__ inline bool row_fast() const { return false; }
    __device__ inline void set_table_ok(bool) {}
    __device__ inline uint32_t col(int64_t j) const { return COMPAT ? 0u : colbase((uint32_t)j); }
    __device__ static inline float pow2(float e) {   // torch.pow(2, e) for integral or +-inf/NaN e
        if (!(fabsf(e) <= 200.f)) return exp2f(e);   // inf -> inf, -inf -> 0, NaN -> NaN
        return ldexpf(1.f, (int)e);                  // exact, incl. subnormal results and 2^128 = inf
    }
    template <bool F>
    __device__ inline float apply(float x, int64_t j, uint32_t cs, const float4*) const {
        const float ax = fabsf(x);
        const float alpha = (float)log2((double)ax);          // correctly rounded fp32 log2
        const float lo = floorf(alpha), hi = ceilf(alpha);
        const float plo = pow2(lo), phi = pow2(hi);
        const float pt = (phi - ax) / plo;
        const bool down = draw_below<COMPAT>(urow, rk, j, cs, hg_of<COMPAT>(rk, j), pt, ldexpf(pt, 32));
        const float out = tsign(x) * (down ? plo : phi);
        return (x == 0.f) ? 0.f : out;
    }
};

// Standard / natural dithering (compressors.py:270-329).  tab[g] = {l[g], l[g+1],
// (l[g]-l[g+1]) * 2^-32, 2^32 / (l[g]-l[g+1])}: the gap is stored pre-scaled so the fast
// division yields p * 2^32 directly (scaling by a power of two commutes with rounding).
// NATBUG: the reference returns (y*sign)*pnorm (its line 326).
template <bool NATBUG, bool COMPAT>
struct DitherOp {
    static constexpr bool TABLE = !NATBUG;
    static constexpr bool HAS_APPLY4 = !NATBUG;
    UniformSrc us;
    RowTabs rt;
    int s;
    float sf;
    FastDiv dn;
    const double* urow;
    uint32_t rk;
    bool fast;
    bool tab_ok;               // every level gap inside the div_fast window (load_table)
    __device__ inline void setup(int64_t row) {
        dn.b = rt.pn[row];
        if (rt.fast) {
            dn.rb = rt.rpn[row];
            dn.ok = fabsf(dn.b) >= 0x1p-40f && fabsf(dn.b) <= 0x1p80f;
            fast = rt.fast[row] && (NATBUG || tab_ok);
        } else {
            dn = make_div(dn.b);
            fast = false;
        }
        urow = COMPAT ? us.u + row * us.uld : nullptr;
        rk = (COMPAT || NATBUG) ? 0u : rt.rk[row];
    }
    __device__ inline bool row_fast() const { return fast; }
    __device__ inline void set_table_ok(bool ok) { tab_ok = ok; }
    __device__ inline uint32_t col(int64_t j) const { return (COMPAT || NATBUG) ? 0u : colbase((uint32_t)j); }
    template <bool F>
    __device__ inline float apply(float x, int64_t j, uint32_t cs, const float4* tab) const {
        // F: the row and the level table are inside the div_fast window (row_fast()); the element
        // path is then branch-free but for the rare one-interval correction of the guess.
        const float ax = fabsf(x);
        const float y = F ? div_fast(ax, dn) : div_rn(ax, dn);                  // |x| / pnorm
        if (NATBUG) return (y * tsign(x)) * dn.b;
        int g = (int)(y * sf);                                 // y >= 0; NaN -> 0
        g = g > s - 1 ? s - 1 : g;
        float4 t = tab[g];
        const bool below = y < t.x, above = y > t.y;
        if (below | above) {                                   // std levels RN(k/s): at most one off
            g = below ? (g > 0 ? g - 1 : 0) : (g < s - 1 ? g + 1 : g);
            t = tab[g];
        }
        const bool in = y <= t.y;                              // y > 1 or NaN: no interval -> 0
        const float num = y - t.y;
        FastDiv dd;
        dd.b = t.z; dd.rb = t.w; dd.ok = true;
        const float p2 = (F || t.w != 0.f) ? div_fast(num, dd) : num / t.z;      // p * 2^32
        const bool down = draw_below<COMPAT>(urow, rk, j, cs, hg_of<COMPAT>(rk, j), COMPAT ? ldexpf(p2, -32) : 0.f, p2);
        const float lev = in ? (down ? t.x : t.y) : 0.f;
        // (lev * sign(x)) * pnorm with out[x == 0] = 0 (compressors.py:294-296)
        return (x == 0.f) ? 0.f : copysignf(lev, x) * dn.b;
    }
    // NE elements, written stage by stage (each step for all elements before the next) so the NE
    // dependency chains are interleaved in the instruction stream; one fix-up branch at the end.
    // uv (compat only, optional): the elements' float64 draws, loaded by the caller ahead of time
    template <bool F, int NE>
    __device__ inline void apply_block(const float* x, const int64_t* jv, const uint32_t* cs, const float4* tab,
                                       float* out, const double* uv = nullptr) const {
        float y[NE], p2[NE];
        float4 t[NE];
        bool fix[NE];
#pragma unroll
        for (int e = 0; e < NE; ++e) y[e] = F ? div_fast(fabsf(x[e]), dn) : div_rn(fabsf(x[e]), dn);
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            int g = (int)(y[e] * sf);
            g = g > s - 1 ? s - 1 : g;
            t[e] = tab[g];
        }
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            fix[e] = (y[e] < t[e].x) | !(y[e] <= t[e].y);
            FastDiv dd;
            dd.b = t[e].z; dd.rb = t[e].w; dd.ok = true;
            const float num = y[e] - t[e].y;
            p2[e] = (F || t[e].w != 0.f) ? div_fast(num, dd) : num / t[e].z;
        }
        bool any = false;
        uint32_t hg[NE / 4];                  // one group hash per aligned 4-element group
#pragma unroll
        for (int c = 0; c < NE / 4; ++c) hg[c] = hg_of<COMPAT>(rk, jv[4 * c]);
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            const bool down = (COMPAT && uv) ? uv[e] < (double)ldexpf(p2[e], -32)
                                             : draw_below<COMPAT>(urow, rk, jv[e], cs[e], hg[e / 4], COMPAT ? ldexpf(p2[e], -32) : 0.f, p2[e]);
            const float lev = down ? t[e].x : t[e].y;
            out[e] = (x[e] == 0.f) ? 0.f : copysignf(lev, x[e]) * dn.b;
            any |= fix[e];
        }
        if (any) {
#pragma unroll
            for (int e = 0; e < NE; ++e)
                if (fix[e]) out[e] = apply<F>(x[e], jv[e], cs[e], tab);
        }
    }
    template <bool F>
    __device__ inline float4 apply4(float4 v, int64_t j, const uint32_t* cs, const float4* tab) const {
        const float x[4] = {v.x, v.y, v.z, v.w};
        const int64_t jv[4] = {j, j + 1, j + 2, j + 3};
        float o[4];
        apply_block<F, 4>(x, jv, cs, tab, o);
        return make_float4(o[0], o[1], o[2], o[3]);
    }
};

template <bool F, class Op>
__device__ inline float4 apply4(const Op& op, float4 v, int64_t j, const uint32_t* cs, const float4* tab) {
    if constexpr (Op::HAS_APPLY4) {
        return op.template apply4<F>(v, j, cs, tab);
    } else {
        return make_float4(op.template apply<F>(v.x, j, cs[0], tab), op.template apply<F>(v.y, j + 1, cs[1], tab),
                           op.template apply<F>(v.z, j + 2, cs[2], tab), op.template apply<F>(v.w, j + 3, cs[3], tab));
    }
}

// COLS float4 groups of one row at once (dithering: one interleaved block, one fix-up branch)
template <bool F, int COLS, class Op>
__device__ inline void apply_cols(const Op& op, const float4* v, const int64_t* gi, const uint32_t (*cs)[4],
                                  const float4* tab, float4* e) {
    if constexpr (Op::HAS_APPLY4) {
        float x[COLS * 4], o[COLS * 4];
        int64_t jv[COLS * 4];
        uint32_t c2[COLS * 4];
#pragma unroll
        for (int c = 0; c < COLS; ++c) {
            x[4 * c] = v[c].x; x[4 * c + 1] = v[c].y; x[4 * c + 2] = v[c].z; x[4 * c + 3] = v[c].w;
#pragma unroll
            for (int q = 0; q < 4; ++q) { jv[4 * c + q] = gi[c] * 4 + q; c2[4 * c + q] = cs[c][q]; }
        }
        op.template apply_block<F, COLS * 4>(x, jv, c2, tab, o);
#pragma unroll
        for (int c = 0; c < COLS; ++c) e[c] = make_float4(o[4 * c], o[4 * c + 1], o[4 * c + 2], o[4 * c + 3]);
    } else {
#pragma unroll
        for (int c = 0; c < COLS; ++c) e[c] = apply4<F>(op, v[c], gi[c] * 4, cs[c], tab);
    }
}

// level table (see DitherOp); returns (block-uniform) whether every gap is inside the window
__device__ inline bool load_table(const float* levels, int s, float4* tab) {
    int bad = 0;
    for (int i = threadIdx.x; i < s; i += blockDim.x) {
        const float lo = levels[i], hi = levels[i + 1], den = lo - hi;
        const float ad = fabsf(den);
        // div_fast window: gap in [2^-40, 2^80] and every nonzero y - hi >= ulp(hi) >= 2^-80
        const bool ok = ad >= 0x1p-40f && ad <= 0x1p80f && hi >= 0x1p-56f;
        const float sden = ldexpf(den, -32);
        tab[i] = make_float4(lo, hi, sden, ok ? 1.0f / sden : 0.f);
        bad |= !ok;
    }
    return __syncthreads_or(bad) == 0;
}


}  // namespace flc
