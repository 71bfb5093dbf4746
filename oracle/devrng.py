"""ORACLE — TEST INFRASTRUCTURE ONLY.  numpy restatement of the build's device-RNG mode.

Device mode is this build's own counter-based generator (the reference draws from numpy's shared
stream instead; compat mode reproduces that bit for bit).  The kernels define it in
flpytorch_amd/csrc/common.hpp (client_key, rowkey, colbase, grouphash, draw_join, dev_u32); this
module states the same arithmetic independently, in vectorised uint32/uint64 numpy, so the
device-mode parity tests do not take their expected draws from the product library:

    ckey  = mix64(seed ^ mix64(0x9E3779B97F4A7C15 * (client + 1)))      (SplitMix64 finaliser)
    rk    = (ckey >> 32) ^ (ckey & 0xFFFFFFFF)
    lo    = fmix32(j * 0x85EBCA77 + (rk ^ 0x27D4EB2F))
    hg    = gmix((j >> 2) * 0x9E3779B1 + rk)                            (one per 4 elements)
    gmix(v): h = v ^ v >> 16; h = mul24(h, 0xB5297B) ^ h >> 24; h ^= h >> 16;
             h = mul24(h, 0x68E31D) ^ h >> 24; h ^ h >> 16      (mul24 = low 32 bits of the
             product of the low 24 bits of each operand)
    u32   = (byte (j & 3) of hg) << 24 | lo >> 8,    u = u32 * 2^-32
"""
import numpy as np

_M64 = (1 << 64) - 1


def _mix64(z):
    z &= _M64
    z ^= z >> 30
    z = (z * 0xBF58476D1CE4E5B9) & _M64
    z ^= z >> 27
    z = (z * 0x94D049BB133111EB) & _M64
    z ^= z >> 31
    return z


def client_key(seed, client):
    return _mix64(int(seed) ^ _mix64((0x9E3779B97F4A7C15 * (int(client) + 1)) & _M64))


def rowkey(ckey):
    return np.uint32(((ckey >> 32) ^ ckey) & 0xFFFFFFFF)


def fmix32(h):
    h = np.asarray(h, dtype=np.uint32).copy()
    h ^= h >> np.uint32(16)
    h *= np.uint32(0x85EBCA6B)
    h ^= h >> np.uint32(13)
    h *= np.uint32(0xC2B2AE35)
    h ^= h >> np.uint32(16)
    return h


def colbase(j):
    return np.asarray(j, dtype=np.uint32) * np.uint32(0x85EBCA77)


def _mul24(a, b):
    return (a & np.uint32(0xFFFFFF)) * np.uint32(b)


def gmix(v):
    """The group hash's mixer (common.hpp gmix, FLC_GHASH 1): two rounds of xorshift + a 24-bit
    multiply with the ignored top byte xored back in."""
    with np.errstate(over="ignore"):
        h = np.asarray(v, dtype=np.uint32).copy()
        h ^= h >> np.uint32(16)
        h = _mul24(h, 0xB5297B) ^ (h >> np.uint32(24))
        h ^= h >> np.uint32(16)
        h = _mul24(h, 0x68E31D) ^ (h >> np.uint32(24))
        return h ^ (h >> np.uint32(16))


def grouphash(g, rk):
    with np.errstate(over="ignore"):
        g = np.asarray(g, dtype=np.uint32)
        return gmix(g * np.uint32(0x9E3779B1) + np.uint32(rk))


def dev_u32(seed, client, j):
    """uint32 draws of one client for element indices j (array)."""
    with np.errstate(over="ignore"):
        j = np.asarray(j, dtype=np.uint32)
        rk = rowkey(client_key(seed, client))
        lo = fmix32(colbase(j) + (rk ^ np.uint32(0x27D4EB2F)))
        hg = grouphash(j >> np.uint32(2), rk)
        top = (hg >> (np.uint32(8) * (j & np.uint32(3)))) & np.uint32(0xFF)
        return (top << np.uint32(24)) | (lo >> np.uint32(8))


def uniforms(seed, client, d):
    """float64 u = u32 * 2^-32 for j = 0..d-1: the `testp` a device-mode encode compares with."""
    return dev_u32(seed, client, np.arange(d, dtype=np.uint32)).astype(np.float64) * (1.0 / 4294967296.0)


# ---------------------------------------------------------------------------------------------
# RandK device sampler (flpytorch_amd/csrc/randk_tree.hpp), restated in numpy integer arithmetic:
#   counts : m_c = #{t < K : Pi(t) in chunk c}, Pi the row permutation of [0, D) (balanced 4-round
#            Feistel on 2h bits, round keys from the client key, cycle-walked into [0, D))
#   members: the first m_c images of a 4-round 6+6-bit Feistel permutation keyed by (client, c)
# ---------------------------------------------------------------------------------------------
_CH = 4096


def row_perm(ckey, d, t):
    """Pi(t) for a uint64 array t (all < d)."""
    b = 1
    while (1 << (2 * b)) < d:
        b += 1
    mask = np.uint64((1 << b) - 1)
    k = _mix64(ckey ^ 0x5851F42D4C957F2D)
    rkey = [np.uint32(_mix64((k + (i << 56)) & _M64) & 0xFFFFFFFF) for i in range(4)]
    sh = np.uint64(b)

    def once(v):
        l = ((v >> sh) & mask).astype(np.uint32)
        r = (v & mask).astype(np.uint32)
        m32 = np.uint32(int(mask))
        for rk in rkey:
            l, r = r, l ^ (fmix32(r ^ rk) & m32)
        return (l.astype(np.uint64) << sh) | r.astype(np.uint64)

    v = once(np.asarray(t, dtype=np.uint64))
    bad = v >= np.uint64(d)
    while bad.any():
        v[bad] = once(v[bad])
        bad = v >= np.uint64(d)
    return v


def randk_counts(seed, client, d, k):
    """Members of the client's device RandK set in each 4096-element chunk (int64[C])."""
    ck = client_key(seed, client)
    C = (d + _CH - 1) // _CH
    v = row_perm(ck, d, np.arange(k, dtype=np.uint64))
    return np.bincount((v >> np.uint64(12)).astype(np.int64), minlength=C).astype(np.int64)


def chunk_perm(ckey, c, clen, t):
    """Images of t (uint32 array) under the chunk permutation of (client key, chunk c), cycle-walked
    into [0, clen)."""
    b = _mix64(ckey ^ ((0xD1B54A32D192ED03 * (c + 1)) & _M64))
    k0, k1 = b & 0xFFFFFFFF, b >> 32
    ks = [np.uint32(k0), np.uint32(k1), fmix32(np.uint32(k0 ^ 0x3C6EF372)),
          fmix32(np.uint32((k1 + 0xA54FF53A) & 0xFFFFFFFF))]

    def once(v):
        l, r = v >> np.uint32(6), v & np.uint32(63)
        for kk in ks:
            l, r = r, l ^ (fmix32(r ^ kk) & np.uint32(63))
        return (l << np.uint32(6)) | r

    v = once(np.asarray(t, dtype=np.uint32))
    bad = v >= clen
    while bad.any():
        v[bad] = once(v[bad])
        bad = v >= clen
    return v


def randk_indices(seed, client, d, k):
    """The client's device-mode RandK index set, chunk by chunk (int64[k])."""
    ck = client_key(seed, client)
    cnt = randk_counts(seed, client, d, k)
    out = []
    for c in np.nonzero(cnt)[0]:
        c = int(c)
        clen = min(_CH, d - c * _CH)
        out.append(c * _CH + chunk_perm(ck, c, clen, np.arange(cnt[c], dtype=np.uint32)).astype(np.int64))
    return np.concatenate(out) if out else np.zeros(0, dtype=np.int64)
