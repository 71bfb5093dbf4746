"""ORACLE — TEST INFRASTRUCTURE ONLY.  numpy restatement of the wire format (flpytorch_amd/csrc/
wire.hip, include/flcodec.h "Wire format"): the payload bytes a row's dense compressVector output
(oracle.codecs.OracleCompressor.compress, pinned to the reference by tests/golden/) packs into.
The reference has no wire format of its own (it counts the bits, compressors.py:223-224, 367-368,
and ships dense tensors, comm_socket.py:16-82): the format is this build's, so these checks pin
the kernels to the stated layout, and the round trip pins it to the reference's outputs.
"""
import numpy as np

from oracle import codecs as oc

F32, Q8, Q16, NAT16, SPARSE, RANKK = 1, 2, 3, 4, 5, 6
_F = np.float32


def _a16(b):
    return (b + 15) & ~15


def payload_format(comp):
    if comp.type == oc.STD_DITHERING:
        return Q8 if comp.s <= 127 else Q16
    if comp.type == oc.NATURAL:
        return NAT16
    if comp.type in (oc.RANDK, oc.TOPK):
        return SPARSE
    if comp.type == oc.RANK_K:
        return RANKK
    return F32


def payload_bytes(comp, d):
    f = payload_format(comp)
    if f == Q8:
        return 16 + _a16(d)
    if f in (Q16, NAT16):
        return 16 + _a16(2 * d)
    if f == SPARSE:
        k = max(1, min(comp.K, d))
        return 16 + 2 * _a16(4 * k)
    if f == RANKK:                       # U'_K (B x K') and (S V'^T)_K' (K' x A), 16-B padded each
        k = min(comp.K, comp.A, comp.B)
        return 16 + _a16(4 * (((comp.B * k + 3) & ~3) + ((k * comp.A + 3) & ~3)))
    return 16 + _a16(4 * d)


def _lev(levels, idx, neg, pn):
    with np.errstate(all="ignore"):
        v = np.where(neg, -levels[idx], levels[idx]).astype(_F)
        return (v * _F(pn)).astype(_F)


def _lev_codes(v, levels, s, pn, sbit):
    vb = v.view(np.uint32)
    neg = (vb >> 31).astype(bool)
    codes = np.zeros(v.size, dtype=np.uint32)
    done = vb == 0
    nan = np.isnan(v)
    codes[nan] = sbit
    done |= nan
    with np.errstate(all="ignore"):
        y = (np.abs(v) / _F(pn)).astype(_F)
        g = np.rint((y * _F(s)).astype(_F)).astype(np.float64)
    g = np.nan_to_num(g, nan=0.0, posinf=s, neginf=0).clip(0, s).astype(np.int64)
    for dlt in (0, -1, 1):
        c = g + dlt
        ok = (~done) & (c >= 0) & (c <= s)
        cc = np.clip(c, 0, s)
        hit = ok & (_lev(levels, cc, neg, pn).view(np.uint32) == vb)
        codes[hit] = np.where(neg[hit], sbit, 0) | cc[hit].astype(np.uint32)
        done |= hit
    bad = 0
    for j in np.nonzero(~done)[0]:                     # binary search, as the kernel
        lo, hi, found = 0, s, None
        while lo <= hi:
            mid = (lo + hi) >> 1
            mv = _lev(levels, np.array([mid]), np.array([neg[j]]), pn)[0]
            if mv.view(np.uint32) == vb[j]:
                found = mid
                break
            if abs(mv) < abs(v[j]):
                lo = mid + 1
            else:
                hi = mid - 1
        if found is None:
            bad += 1
            codes[j] = sbit if neg[j] else 0
        else:
            codes[j] = (sbit if neg[j] else 0) | found
    return codes, bad


def _nat_codes(v):
    vb = v.view(np.uint32)
    sg = ((vb >> 31) << 15).astype(np.uint32)
    codes = sg.copy()
    mag = vb & 0x7FFFFFFF
    nan = np.isnan(v)
    inf = np.isinf(v)
    reg = (mag != 0) & ~nan & ~inf
    _, e = np.frexp(v[reg])
    codes[reg] = sg[reg] | (e.astype(np.int64) - 1 + 16384).astype(np.uint32)
    codes[inf] = sg[inf] | 0x7FFE
    codes[nan] = 0x7FFF
    return codes


def pack(comp, out, pnorm=None):
    """Payload bytes (uint8 array) of one row's dense output `out` under compressor `comp`."""
    out = np.asarray(out, dtype=_F)
    d = out.size
    f = payload_format(comp)
    if f == RANKK:
        raise NotImplementedError("rank_k payloads hold the SVD factors; their signs are the solver's own")
    buf = np.zeros(payload_bytes(comp, d), dtype=np.uint8)
    hdr = np.zeros(4, dtype=np.uint32)
    hdr[0] = f
    if f == SPARSE:
        k = max(1, min(comp.K, d))
        nz = np.nonzero(out.view(np.uint32) != 0)[0]
        hdr[1] = nz.size
        hdr[3] = max(0, nz.size - k)
        nz = nz[:k]
        buf[16:16 + 4 * nz.size] = nz.astype(np.uint32).view(np.uint8)
        o = 16 + _a16(4 * k)
        buf[o:o + 4 * nz.size] = out[nz].view(np.uint8)
    elif f in (Q8, Q16):
        hdr[1] = d
        hdr[2] = np.array([pnorm], dtype=_F).view(np.uint32)[0]
        sbit = 0x80 if f == Q8 else 0x8000
        codes, bad = _lev_codes(out, comp.levels, comp.s, pnorm, sbit)
        hdr[3] = bad
        body = codes.astype(np.uint8 if f == Q8 else np.uint16).view(np.uint8)
        buf[16:16 + body.size] = body
    elif f == NAT16:
        hdr[1] = d
        body = _nat_codes(out).astype(np.uint16).view(np.uint8)
        buf[16:16 + body.size] = body
    else:
        hdr[1] = d
        buf[16:16 + 4 * d] = out.view(np.uint8)
    buf[:16] = hdr.view(np.uint8)
    return buf


def unpack(comp, payload, d):
    """Dense fp32 row of a payload (the restated decode)."""
    payload = np.asarray(payload, dtype=np.uint8)
    hdr = payload[:16].view(np.uint32)
    f, cnt = int(hdr[0]), int(hdr[1])
    norm = payload[8:12].view(_F)[0]
    body = payload[16:]
    if f == SPARSE:
        k = max(1, min(comp.K, d))
        cnt = min(cnt, k)
        idx = body[:4 * cnt].view(np.uint32)
        o = _a16(4 * k)
        val = body[o:o + 4 * cnt].view(_F)
        out = np.zeros(d, dtype=_F)
        out[idx] = val
        return out
    if f == F32:
        return body[:4 * d].view(_F).copy()
    if f == NAT16:
        c = body[:2 * d].view(np.uint16).astype(np.uint32)
        m = c & 0x7FFF
        sg = np.where(c & 0x8000, _F(-1), _F(1))
        with np.errstate(all="ignore"):
            v = np.ldexp(_F(1), (m.astype(np.int64) - 16384).clip(-200, 200).astype(np.int32)).astype(_F)
        v = np.where(m == 0, _F(0), v)
        v = np.where(m == 0x7FFE, _F(np.inf), v)
        v = np.copysign(v, sg).astype(_F)
        v[m == 0x7FFF] = np.nan
        return v
    sbit = 0x80 if f == Q8 else 0x8000
    c = (body[:d] if f == Q8 else body[:2 * d].view(np.uint16)).astype(np.int64)
    idx = c & (sbit - 1)
    neg = (c & sbit) != 0
    v = _lev(comp.levels, idx, neg, norm)
    v[c == 0] = _F(0)
    return v
