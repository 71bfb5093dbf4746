"""ORACLE — TEST INFRASTRUCTURE ONLY.

numpy restatement of the reference codecs and reduction, op for op in fp32:

* ``parse_spec`` / ``OracleCompressor.__init__``  — initCompressor, compressors.py:435-494,
  and the make* constructors, compressors.py:64-178.
* ``OracleCompressor.generate``  — generateCompressPattern, compressors.py:196-216.
* ``OracleCompressor.compress``  — compressVector, compressors.py:218-371 (rank_k: numpy's float32
  LAPACK SVD, like torch's CPU path; its outputs match the reference to a tolerance, not bits).
* ``server_gradient``            — serverGradient core, algorithms.py:1748-1770 (DCGD) and
  1810-1832 (FedAvg): gs = w0 (x - x0); gs += wi (x - xi) in buffer order; gs / sum(w).
* ``reduce_plain``               — the fused encode+reduce contract of the product:
  the same sequential fp32 sum over already-encoded rows (sum_i wi * C(g_i)) / sum(w).

fp32 semantics reproduced (checked against tests/golden/ fixtures from the real reference):
  * python-float scalars multiply / divide fp32 tensors as fp32 scalars (torch CPU rule);
  * dithering compares the float64 uniforms with the fp32 probability promoted to float64
    (compressors.py:288);  later level intervals overwrite earlier ones (290-291);
  * ``out * sign * pnorm`` is evaluated left to right in fp32 (296);
  * natural dithering returns ``y * sign * pnorm`` — the reference's own bug (326);
  * torch's CPU ``norm`` sums in its own fp32 order (14 616 ulp from the exact value at
    D = 25 M); the oracle computes the norm exactly (float64 accumulation, one rounding) unless
    the caller passes a value — the reference's, or oracle/torch_norm.c's restatement of torch's
    order (the library's norm_mode="torch_cpu").
  * TopK ties at the K-th magnitude are broken by lowest index (torch leaves it unspecified);
    ``tie = "highest"`` keeps the highest indices instead (the library's FLC_TIE_HIGHEST).
"""
import math

import numpy as np

IDENTICAL, LAZY, RANDK, NATURAL, STD_DITHERING, NAT_DITHERING, TOPK, RANK_K = range(1, 9)
_F32 = np.float32


def _levels_std(levels):
    # torch.arange(0.0, 1.0 + 1.0/levels*0.5, 1.0/levels) (compressors.py:87).  The reference's
    # own call, on the CPU: torch's vectorised arange forms start + step * i partly in fp32, so a
    # float64 restatement differs from it in the last bit for s >= ~300 (s = 300: 259 of 4099
    # QSGD outputs one ulp apart).  The call is deterministic third-party arithmetic, pinned by the
    # golden level tables (tests/test_oracle_golden.py::test_codec_constants).
    import torch
    return torch.arange(0.0, 1.0 + 1.0 / levels * 0.5, 1.0 / levels, dtype=torch.float32).numpy().copy()


def _levels_nat(levels):
    # compressors.py:116-119: zeros(levels+1); [i] = 0.5**i for i < levels; flip.
    v = np.zeros(levels + 1, dtype=_F32)
    for i in range(levels):
        v[i] = _F32(0.5 ** i)
    return v[::-1].copy()


class OracleCompressor:
    def __init__(self, spec, D):
        params = spec.split(":")
        name = params[0]
        self.D = D
        self.K = None
        self.testp = None
        self.S = None
        self.total_input_components = 0
        self.really_need_to_send_components = 0
        self.last_input_advance = 0
        self.last_need_to_send_advance = 0
        self.tie = "lowest"          # TopK tie rule (the library's flc_codec_params.tie)

        def kspec(arg):
            if arg.find("%") == -1:
                return math.ceil(float(arg))
            return math.ceil(float(arg[0:-1]) / 100.0 * D)

        def pspec():
            if len(params) == 3:
                return math.inf if params[2].lower() == "inf" else int(params[2])
            return math.inf

        if name == "ident":
            self.type, self.w = IDENTICAL, 0.0
        elif name == "randk":
            self.type, self.K = RANDK, kspec(params[1])
            self.w = D / self.K - 1.0
        elif name == "bernulli":
            self.type, self.P = LAZY, float(params[1])
            self.w = 1.0 / self.P - 1.0
        elif name == "natural":
            self.type, self.w = NATURAL, 1.0 / 8.0
        elif name in ("qsgd", "std.dithering", "terngrad"):
            if name == "terngrad":
                L, p = 1, math.inf
            elif name == "qsgd":
                L, p = int(params[1]), 2
            else:
                L, p = int(params[1]), pspec()
            self.type = STD_DITHERING
            self.levels = _levels_std(L)
            self.s = len(self.levels) - 1
            assert self.s == L
            self.p = p
            if name == "qsgd":
                self.w = min(D / (L * L), D ** 0.5 / L)
            else:
                self.w = 0.0
        elif name == "nat.dithering":
            L, p = int(params[1]), pspec()
            self.type = NAT_DITHERING
            self.levels = _levels_nat(L)
            self.s = L
            self.p = p
            r = min(p, 2)
            self.w = 1.0 / 8.0 + (D ** (1.0 / r)) / (2 ** (self.s - 1)) * min(1, (D ** (1.0 / r)) / (2 ** (self.s - 1)))
        elif name == "topk":
            self.type, self.K = TOPK, kspec(params[1])
            self.alpha = self.K / D
        elif name == "rank_k":                        # makeRankKCompressor, compressors.py:151-172
            self.type, self.K = RANK_K, kspec(params[1])
            a = int(D ** 0.5)
            while D % a != 0:
                a += 1
            self.A, self.B = a, D // a
            self.alpha = self.K / min(self.A, self.B)
        else:
            raise AssertionError("Unknown compressor format")   # compressors.py:492

    # compressors.py:196-216
    def generate(self, rs):
        t = self.type
        if t == LAZY:
            self.testp = rs.random()
        elif t == RANDK:
            self.S = rs.choice(self.D, self.K, replace=False)
        elif t in (NATURAL, STD_DITHERING, NAT_DITHERING):
            self.testp = rs.rand(self.D)

    def norm(self, x):
        if self.p == math.inf:
            return _F32(np.max(np.abs(x))) if x.size else _F32(0)
        if self.p == 2:
            return _F32(np.sqrt(np.sum(x.astype(np.float64) ** 2)))
        if self.p == 1:
            return _F32(np.sum(np.abs(x).astype(np.float64)))
        return _F32(np.sum(np.abs(x).astype(np.float64) ** self.p) ** (1.0 / self.p))

    # compressors.py:218-371
    def compress(self, x, pnorm=None):
        x = np.asarray(x, dtype=_F32)
        d = max(x.shape)
        t = self.type
        need = 0
        with np.errstate(all="ignore"):
            if t == IDENTICAL:
                out, need = x, d
            elif t == LAZY:
                if self.testp < self.P:
                    out, need = x / _F32(self.P), d
                else:
                    out, need = np.zeros_like(x), 0
            elif t == RANDK:
                out = np.zeros_like(x)
                out[self.S] = _F32(self.D / self.K) * x[self.S]
                need = self.K
            elif t == NATURAL:
                out = np.zeros_like(x)
                sign = np.sign(x)
                ax = np.abs(x)
                alpha = np.log2(ax)
                lo, hi = np.floor(alpha), np.ceil(alpha)
                p_lo, p_hi = np.exp2(lo), np.exp2(hi)
                pt = (p_hi - ax) / p_lo
                down = self.testp < pt.astype(np.float64)
                out[down] = (sign * p_lo)[down]
                out[~down] = (sign * p_hi)[~down]
                out[x == 0.0] = 0.0
                need = 9.0 / 32.0 * d
            elif t in (STD_DITHERING, NAT_DITHERING):
                pn = self.norm(x) if pnorm is None else _F32(pnorm)
                sign = np.sign(x)
                y = np.abs(x) / pn
                lv = self.levels
                u = self.testp
                if d <= LOOP_MAX_D:
                    out = np.zeros_like(x)
                    for s in range(len(lv) - 1):
                        c12 = (y >= lv[s]) & (y <= lv[s + 1])
                        p = (y - lv[s + 1]) / (lv[s] - lv[s + 1])
                        c3 = u < p.astype(np.float64)
                        out[c12 & c3] = lv[s]
                        out[c12 & ~c3] = lv[s + 1]
                else:
                    out = dither_levels(y, u, lv)
                out[x == 0.0] = 0.0
                if t == STD_DITHERING:
                    out = out * sign * pn
                else:
                    out = y * sign * pn
                need = 1.0 + d * (1.0 + math.ceil(math.log2(self.s))) / 32.0
            elif t == TOPK:
                out = np.zeros_like(x)
                ind = topk_indices(x, self.K, self.tie)
                out[ind] = x[ind]
                need = self.K
            elif t == RANK_K:                         # compressors.py:336-364
                U, S, Vt = np.linalg.svd(x.reshape(self.A, self.B), full_matrices=False)
                K = min(len(S), self.K)
                out = ((U[:, :K] * S[:K]) @ Vt[:K, :]).astype(_F32).reshape(d)
                need = K * (self.A + self.B)
            else:
                raise NotImplementedError(f"codec {t}")
        self.last_input_advance = d
        self.last_need_to_send_advance = need
        self.really_need_to_send_components += need
        self.total_input_components += d
        return out


# Above this D the dithering level loop (O(s D) numpy passes, compressors.py:284-291) is replaced by
# dither_levels, its closed form; tests/test_oracle_golden.py pins the two equal.
LOOP_MAX_D = 1 << 20


def dither_levels(y, u, lv):
    """Closed form of the reference's level loop (compressors.py:284-291) in one pass.

    The loop visits the intervals s = 0..S-1 in order and assigns to every element with
    lv[s] <= y <= lv[s+1]; an element on a level boundary lies in two intervals and the LATER one
    wins, so the effective interval is the largest s with lv[s] <= y, clipped to S-1 when
    y == lv[S]; y above lv[S] (or NaN) lies in none and stays 0.  Inside it the same fp32
    arithmetic: p = (y - lv[s+1]) / (lv[s] - lv[s+1]), lv[s] if u < p (float64 compare) else lv[s+1]."""
    S = len(lv) - 1
    s = np.searchsorted(lv, y, side="right").astype(np.int64) - 1
    inside = (s >= 0) & ((s < S) | (y == lv[S]))
    s = np.clip(s, 0, S - 1)
    lo, hi = lv[s], lv[s + 1]
    p = (y - hi) / (lo - hi)
    out = np.where(u < p.astype(np.float64), lo, hi).astype(_F32)
    out[~inside] = 0.0
    return out


def topk_keys(x):
    """Order-preserving uint32 key of |x| (NaN above +inf, like torch.topk)."""
    return (np.asarray(x, dtype=_F32).view(np.uint32) & np.uint32(0x7FFFFFFF))


def topk_indices(x, K, tie="lowest"):
    """Indices of the K largest |x|, ties at the K-th magnitude broken by lowest index
    (compressors.py:330-335 with torch.topk's CPU tie order) or, tie="highest", by highest index
    (the library's FLC_TIE_HIGHEST)."""
    key = topk_keys(x).astype(np.int64)
    pos = np.arange(key.size) if tie == "lowest" else -np.arange(key.size)
    order = np.lexsort((pos, -key))
    return np.sort(order[:K])


def topk_indices_fast(x, K, tie="lowest"):
    """topk_indices by selection instead of a full sort (same set; large rows in the GPU tests):
    every key above the K-th key, then the lowest- (or highest-) index keys equal to it."""
    key = topk_keys(x)
    K = int(K)
    if K <= 0:
        return np.empty(0, dtype=np.int64)
    if K >= key.size:
        return np.arange(key.size, dtype=np.int64)
    kth = np.partition(key, key.size - K)[key.size - K]
    above = np.flatnonzero(key > kth)
    eq = np.flatnonzero(key == kth)
    ties = eq[:K - above.size] if tie == "lowest" else eq[eq.size - (K - above.size):]
    return np.sort(np.concatenate([above, ties])).astype(np.int64)


def server_gradient(x, models, weights=None):
    """algorithms.py:1753-1768: sequential fp32, python-float weights applied as fp32."""
    x = np.asarray(x, dtype=_F32)
    n = len(models)
    if n == 0:
        return np.zeros_like(x)                          # algorithms.py:2117-2118
    w = [1.0] * n if weights is None else [float(v) for v in weights]
    gs = _F32(w[0]) * (x - np.asarray(models[0], dtype=_F32))
    wt = w[0]
    for i in range(1, n):
        gi = x - np.asarray(models[i], dtype=_F32)
        wt += w[i]
        gs = gs + _F32(w[i]) * gi
    return gs / _F32(wt)


def reduce_plain(rows, weights=None):
    """(sum_i w_i * row_i) / sum(w), sequential fp32 in row order (fused encode+reduce contract)."""
    n = len(rows)
    w = [1.0] * n if weights is None else [float(v) for v in weights]
    gs = _F32(w[0]) * np.asarray(rows[0], dtype=_F32)
    wt = w[0]
    for i in range(1, n):
        wt += w[i]
        gs = gs + _F32(w[i]) * np.asarray(rows[i], dtype=_F32)
    return gs / _F32(wt)


def shift_step(comp, a, b, scale=1.0, base=None, alpha=None, h=None, pnorm=None):
    """The shift codecs' client step, fp32 op for op as the torch expressions:
    e = C(a - b); msg = base + e * scale (e * scale without base); h' = h + alpha * e.
    DIANA algorithms.py:1383-1391 (scale 1, no base, h += alpha m), EF21 1506-1517
    (base = b = g_prev, scale = 1 / (1 + w) or 1), MARINA 537 / 691 (base = g_prev),
    FRECON 1104-1110, COFIG 1265-1269.  Python scalars enter as fp32 (torch's tensor-scalar ops)."""
    with np.errstate(all="ignore"):
        diff = (np.asarray(a, dtype=_F32) - np.asarray(b, dtype=_F32)).astype(_F32)
        e = comp.compress(diff, pnorm=pnorm)
        t = (e * _F32(scale)).astype(_F32)
        msg = t if base is None else (np.asarray(base, dtype=_F32) + t).astype(_F32)
        h2 = None
        if alpha is not None:
            h2 = (np.asarray(h, dtype=_F32) + (_F32(alpha) * e).astype(_F32)).astype(_F32)
    return msg, h2
