"""ORACLE — TEST INFRASTRUCTURE ONLY.  numpy restatement of the build's device-RNG mode.

Device mode is this build's own counter-based generator (the reference draws from numpy's shared
stream instead; compat mode reproduces that bit for bit).  The kernels define it in
flpytorch_amd/csrc/common.hpp (client_key, rowkey, colbase, grouphash, draw_join, dev_u32); this
module states the same arithmetic independently, in vectorised uint32/uint64 numpy, so the
device-mode parity tests do not take their expected draws from the product library:

    ckey  = mix64(seed ^ mix64(0x9E3779B97F4A7C15 * (client + 1)))      (SplitMix64 finaliser)
    rk    = (ckey >> 32) ^ (ckey & 0xFFFFFFFF)
    lo    = fmix32(j * 0x85EBCA77 + (rk ^ 0x27D4EB2F))
    hg    = fmix32((j >> 2) * 0x9E3779B1 + rk)                          (one per 4 elements)
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


def grouphash(g, rk):
    g = np.asarray(g, dtype=np.uint32)
    return fmix32(g * np.uint32(0x9E3779B1) + np.uint32(rk))


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
