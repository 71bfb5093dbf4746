"""ORACLE — TEST INFRASTRUCTURE ONLY.  ctypes front-end of oracle/mt19937_legacy.c.

Restates the numpy legacy ``RandomState`` calls FL_PyTorch makes on its shared experiment
stream (execution_context.py:25):
  choice(D, K, replace=False)  compressors.py:206 ; fl_funcs.py:15
  rand(D)                      compressors.py:208-212
  random()                     compressors.py:204
  randint(2**31)               algorithms.py:2055
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle_rng.so")
_lib = None


def _load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    lib = ctypes.CDLL(_LIB_PATH)
    vp, i64, u32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint32
    lib.orc_mt_seed.argtypes = [vp, u32]
    lib.orc_mt_next32.argtypes = [vp]
    lib.orc_mt_next32.restype = u32
    lib.orc_mt_next_double.argtypes = [vp]
    lib.orc_mt_next_double.restype = ctypes.c_double
    lib.orc_mt_choice.argtypes = [vp, i64, i64, vp, vp]
    lib.orc_mt_rand.argtypes = [vp, i64, vp]
    lib.orc_mt_randint31.argtypes = [vp]
    lib.orc_mt_randint31.restype = i64
    lib.orc_mt_state_size.restype = ctypes.c_int
    _lib = lib
    return lib


class OracleRandomState:
    """Subset of numpy.random.RandomState (legacy) the reference's hot path uses."""

    def __init__(self, seed):
        lib = _load()
        self._buf = ctypes.create_string_buffer(lib.orc_mt_state_size())
        lib.orc_mt_seed(self._buf, ctypes.c_uint32(int(seed) & 0xFFFFFFFF))

    @property
    def _p(self):
        return ctypes.cast(self._buf, ctypes.c_void_p)

    def choice(self, n, k, replace=False):
        assert not replace
        out = np.empty(k, dtype=np.int64)
        perm = np.empty(max(n, 1), dtype=np.int64)
        _lib.orc_mt_choice(self._p, n, k, out.ctypes.data, perm.ctypes.data)
        return out

    def rand(self, n):
        out = np.empty(n, dtype=np.float64)
        _lib.orc_mt_rand(self._p, n, out.ctypes.data)
        return out

    def random(self):
        return _lib.orc_mt_next_double(self._p)

    def randint31(self):
        return int(_lib.orc_mt_randint31(self._p))

    def next32(self):
        return int(_lib.orc_mt_next32(self._p))

    def state(self):
        """(key[624] uint32, pos) — same layout as numpy's get_state()[1:3]."""
        raw = np.frombuffer(self._buf.raw, dtype=np.uint32)
        return raw[:624].copy(), int(np.frombuffer(self._buf.raw[624 * 4:624 * 4 + 4], dtype=np.int32)[0])
