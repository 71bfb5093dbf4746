"""Drop-in ``Compressor`` for FL_PyTorch's codec protocol, executed on MI355X.

Mirrors the object protocol of ``fl_pytorch/utils/compressors.py`` — the factory
``initCompressor(spec, D)`` (435-494), the ``make*`` constructors and constants (64-194),
``generateCompressPattern(rndgen, device, clientId, H)`` (196-216), ``compressVector(x)``
(218-371) and the wire-size statistics (25-38, 223-224, 367-368) — so the reference's algorithm
classes and ``run.py`` drive it unchanged (see ``flpytorch_amd.aggregation.install``).

Where the work runs
-------------------
* Patterns (compat mode, the default) are drawn from the caller's own ``np.random.RandomState``
  by libflcodec's host MT19937 (``flc_mt_*``): the state is read with ``get_state()``, advanced
  in C++ exactly as numpy would advance it, and written back with ``set_state()`` — the shared
  experiment stream stays bit-identical to the reference's.
* Encoding always runs in the HIP kernels of libflcodec.so (``flc_encode``).  A host tensor is
  copied to the GPU and the result copied back (the simulator's end-to-end path); with no HIP
  device visible the call raises — there is no CPU implementation in the product.

Error behaviour follows the reference: an unknown spec raises ``AssertionError`` (492); a
non-fp32 input raises ``TypeError`` (the kernels are fp32-only).
"""
import ctypes
import math

import numpy as np
import torch

from .. import _lib


class CompressorType:
    """Same ids as the reference (compressors.py:11-19) and the C ABI's flc_codec."""
    IDENTICAL = 1
    LAZY_COMPRESSOR = 2
    RANDK_COMPRESSOR = 3
    NATURAL_COMPRESSOR_FP32 = 4
    STANDARD_DITHERING_FP32 = 5
    NATURAL_DITHERING_FP32 = 6
    TOPK_COMPRESSOR = 7
    RANK_K_COMPRESSOR = 8


_OMEGA = r'$\omega$'


# ---------------------------------------------------------------------------------------------
# numpy legacy stream, advanced by libflcodec (bit-identical to RandomState's own draws)
# ---------------------------------------------------------------------------------------------
class _StreamState:
    """Borrow a RandomState's MT19937 state for libflcodec; ``commit`` hands it back."""

    def __init__(self, rndgen):
        st = rndgen.get_state()
        if st[0] != "MT19937":
            raise TypeError("generateCompressPattern: rndgen must be a numpy RandomState (MT19937)")
        self.rndgen = rndgen
        self.key = np.array(st[1], dtype=np.uint32, copy=True)
        self.pos = np.array([st[2]], dtype=np.int32)
        self.gauss = (st[3], st[4])

    def ptrs(self):
        return ctypes.c_void_p(self.key.ctypes.data), ctypes.c_void_p(self.pos.ctypes.data)

    def commit(self):
        self.rndgen.set_state(("MT19937", self.key, int(self.pos[0]), self.gauss[0], self.gauss[1]))


def stream_choice(rndgen, n, k):
    """== rndgen.choice(n, k, replace=False) (numpy legacy), drawn by libflcodec."""
    lib = _lib.load()
    s = _StreamState(rndgen)
    out = np.empty(k, dtype=np.int64)
    scratch = np.empty(max(n, 1), dtype=np.int64)
    _lib.check(lib.flc_mt_choice(*s.ptrs(), n, k, out.ctypes.data, scratch.ctypes.data), "flc_mt_choice")
    s.commit()
    return out


def stream_rand(rndgen, n, out=None):
    """== rndgen.rand(n) (float64), drawn by libflcodec into `out` (e.g. pinned host memory)."""
    lib = _lib.load()
    s = _StreamState(rndgen)
    if out is None:
        out = np.empty(n, dtype=np.float64)
    _lib.check(lib.flc_mt_rand(*s.ptrs(), n, out.ctypes.data), "flc_mt_rand")
    s.commit()
    return out


def stream_random(rndgen):
    """== rndgen.random()."""
    return float(stream_rand(rndgen, 1)[0])


def stream_randint31(rndgen, count=1):
    """== [rndgen.randint(2**31) for _ in range(count)]."""
    lib = _lib.load()
    s = _StreamState(rndgen)
    out = np.empty(count, dtype=np.int64)
    _lib.check(lib.flc_mt_randint31(*s.ptrs(), count, out.ctypes.data), "flc_mt_randint31")
    s.commit()
    return out


# ---------------------------------------------------------------------------------------------
# Level tables — built with the same torch calls as the reference so the fp32 values match
# ---------------------------------------------------------------------------------------------
def std_levels(levels):
    return torch.arange(0.0, 1.0 + 1.0 / levels * 0.5, 1.0 / levels)          # compressors.py:87


def nat_levels(levels):
    v = torch.zeros(levels + 1)                                               # compressors.py:116-119
    v[:levels] = torch.tensor([(1.0 / 2.0) ** i for i in range(levels)])
    return torch.flip(v, dims=[0])


def _gpu_device(x):
    _lib.require_gpu()
    if x.is_cuda:
        return x.device
    return torch.device("cuda", torch.cuda.current_device())


class Compressor:
    """Unbiased / contractive gradient codecs (E[C(x)] = x, E|C(x)-x|^2 <= w|x|^2, or top-K)."""

    # -- statistics (compressors.py:25-38) -------------------------------------------------
    def resetStats(self):
        self.total_input_components = 0
        self.really_need_to_send_components = 0
        self.last_input_advance = 0
        self.last_need_to_send_advance = 0

    def __init__(self):
        self.compressorType = CompressorType.IDENTICAL
        self.resetStats()
        self.device_rng = None   # (seed, client) -> device counter-based patterns (opt-in)
        # execution hints (flc_codec_params.flags); results are identical for every setting:
        #   dither_path  None | "sparse" | "dense"  (QSGD p=2 fused uplink, device-RNG or compat draws)
        #   row_groups   None | g                   (folds pipelined under the next group's pass)
        self.dither_path = None
        self.row_groups = None
        # what (not how): the p = 2 norm of standard dithering / QSGD in compressVector —
        #   "exact"      the correctly rounded norm (default; deterministic on every host)
        #   "torch_cpu"  the reference's own fp32 value, torch.norm(x, p=2) on a CPU tensor
        #                (compressors.py:272 / 303: standard and natural dithering) in torch's CPU
        #                reduction order, bit for bit on x86 hosts with AVX2 (torch's 8-lane AVX2
        #                norm kernel, which AVX512 hosts run too; without AVX2: unpinned)
        #                (flc_norm2_torch_cpu; latency-bound: see bench.py --dropin --norm-mode)
        self.norm_mode = "exact"
        # what: TopK's choice among entries tied at the K-th magnitude when fewer places are left
        # than ties (compressors.py:332 leaves it to torch.topk) — "lowest" indices (default: the
        # order torch.topk's CPU kernel gave on the reference's rows) or "highest" (flc_codec_params.tie)
        self.tie_policy = "lowest"

    # -- constants -------------------------------------------------------------------------
    def fullName(self):
        t = self.compressorType
        if t == CompressorType.IDENTICAL:
            return "Identical"
        if t == CompressorType.LAZY_COMPRESSOR:
            return f"Bernoulli(Lazy) [p={self.P:g},{_OMEGA}={self.getW():.1f}]"
        if t == CompressorType.RANDK_COMPRESSOR:
            return f"Rand [K={self.K},D={self.D}]"
        if t == CompressorType.NATURAL_COMPRESSOR_FP32:
            return f"Natural for fp32 [{_OMEGA}={self.getW():.1f}]"
        if t == CompressorType.STANDARD_DITHERING_FP32:
            return f"Standard Dithering for fp32[s={self.s}]"
        if t == CompressorType.NATURAL_DITHERING_FP32:
            return f"Natural Dithering for fp32[s={self.s},{_OMEGA}={self.getW():.1f}]"
        if t == CompressorType.TOPK_COMPRESSOR:
            return f"Top [K={self.K},D={self.D}]"
        if t == CompressorType.RANK_K_COMPRESSOR:
            return f"Rank [K={self.K},D={self.D}]"
        return "?"

    def makeIdenticalCompressor(self):
        self.compressorType = CompressorType.IDENTICAL
        self.w = 0.0
        self.resetStats()

    def makeLazyCompressor(self, P):
        self.compressorType = CompressorType.LAZY_COMPRESSOR
        self.P = P
        self.w = 1.0 / P - 1.0
        self.resetStats()

    def makeStandardDitheringFP32(self, D, levels, p=float("inf")):
        self.D = D
        self.compressorType = CompressorType.STANDARD_DITHERING_FP32
        self.levelsValues = std_levels(levels)
        self.s = len(self.levelsValues) - 1
        assert self.s == levels
        self.p = p
        self.w = 0.0
        self.resetStats()

    def makeQSGD_FP32(self, D, levels):
        self.makeStandardDitheringFP32(D, levels, p=2)
        self.w = min(D / (levels * levels), D ** 0.5 / levels)   # QSGD Lemma 3.1

    def makeTernGrad(self, D):
        self.makeStandardDitheringFP32(D, levels=1, p=float("inf"))
        self.w = 0.0

    def makeNaturalDitheringFP32(self, D, levels, p=float("inf")):
        self.D = D
        self.compressorType = CompressorType.NATURAL_DITHERING_FP32
        self.levelsValues = nat_levels(levels)
        self.s = len(self.levelsValues) - 1
        assert self.s == levels
        self.p = p
        r = min(p, 2)
        self.w = 1.0 / 8.0 + (D ** (1.0 / r)) / (2 ** (self.s - 1)) * min(1, (D ** (1.0 / r)) / (2 ** (self.s - 1)))
        self.resetStats()

    def makeRandKCompressor(self, D, K):
        self.compressorType = CompressorType.RANDK_COMPRESSOR
        self.K = K
        self.D = D
        self.w = self.D / self.K - 1.0
        self.resetStats()

    def makeTopKCompressor(self, D, K):
        self.compressorType = CompressorType.TOPK_COMPRESSOR
        self.K = K
        self.D = D
        self.alpha = self.K / self.D
        self.resetStats()

    def makeRankKCompressor(self, D, K):
        self.compressorType = CompressorType.RANK_K_COMPRESSOR
        self.K = K
        self.D = D
        a = int(D ** 0.5)
        while self.D % a != 0:
            a += 1
        self.A, self.B = a, self.D // a
        self.alpha = self.K / min(self.A, self.B)
        self.resetStats()

    def makeNaturalCompressorFP32(self, D):
        self.compressorType = CompressorType.NATURAL_COMPRESSOR_FP32
        self.D = D
        self.w = 1.0 / 8.0
        self.resetStats()

    def getW(self):
        return self.w

    def getAlphaContraction(self):
        return self.alpha

    def isContractionCompressor(self):
        return hasattr(self, "alpha")

    def isUnbiasedCompressor(self):
        return hasattr(self, "w")

    # -- patterns (compressors.py:196-216) ---------------------------------------------------
    def generateCompressPattern(self, rndgen, device, clientId, H):
        t = self.compressorType
        if t == CompressorType.LAZY_COMPRESSOR:
            self.testp = stream_random(rndgen)
        elif t == CompressorType.RANDK_COMPRESSOR:
            self.S = torch.from_numpy(stream_choice(rndgen, self.D, self.K)).to(torch.long).to(device=device)
        elif t in (CompressorType.NATURAL_COMPRESSOR_FP32, CompressorType.STANDARD_DITHERING_FP32,
                   CompressorType.NATURAL_DITHERING_FP32):
            pin = torch.cuda.is_available()
            buf = torch.empty(self.D, dtype=torch.float64, pin_memory=pin)
            stream_rand(rndgen, self.D, out=buf.numpy())
            self.testp = buf

    # -- encode (compressors.py:218-371) -----------------------------------------------------
    def codec_params(self, device):
        """flc_codec_params for this compressor (levels uploaded to `device`)."""
        t = self.compressorType
        prm = _lib.FlcCodecParams()
        prm.codec = int(t)
        if t in (CompressorType.RANDK_COMPRESSOR, CompressorType.TOPK_COMPRESSOR, CompressorType.RANK_K_COMPRESSOR):
            prm.k = int(self.K)
        if t == CompressorType.RANDK_COMPRESSOR:
            prm.randk_scale = float(np.float32(self.D / self.K))
        if t == CompressorType.LAZY_COMPRESSOR:
            prm.lazy_p = float(np.float32(self.P))
        keep = []
        if t in (CompressorType.STANDARD_DITHERING_FP32, CompressorType.NATURAL_DITHERING_FP32):
            if self.levelsValues.device != device:
                self.levelsValues = self.levelsValues.to(device=device)
            prm.s = int(self.s)
            norms = {1: _lib.FLC_NORM_L1, 2: _lib.FLC_NORM_L2, math.inf: _lib.FLC_NORM_LINF}
            if self.p not in norms:
                raise NotImplementedError(f"p-norm {self.p}: flcodec implements p in (1, 2, inf)")
            prm.norm = norms[self.p]
            prm.d_levels = self.levelsValues.data_ptr()
            keep.append(self.levelsValues)
        if self.device_rng is not None:
            prm.seed = int(self.device_rng[0]) & 0xFFFFFFFFFFFFFFFF
        flags = {None: _lib.FLC_PATH_AUTO, "sparse": _lib.FLC_PATH_SPARSE, "dense": _lib.FLC_PATH_DENSE}
        if getattr(self, "dither_path", None) not in flags:
            raise ValueError(f"dither_path must be None, 'sparse' or 'dense' (got {self.dither_path!r})")
        prm.flags = flags[getattr(self, "dither_path", None)]
        if getattr(self, "row_groups", None):
            prm.flags |= _lib.FLC_ROW_GROUPS(self.row_groups)
        ties = {"lowest": _lib.FLC_TIE_LOWEST, "highest": _lib.FLC_TIE_HIGHEST}
        if getattr(self, "tie_policy", "lowest") not in ties:
            raise ValueError(f"tie_policy must be 'lowest' or 'highest' (got {self.tie_policy!r})")
        prm.tie = ties[getattr(self, "tie_policy", "lowest")]
        return prm, keep

    def _need_to_send(self, d):
        """Wire count of one call (compressors.py:227-364, the last_need_to_send_advance lines)."""
        t = self.compressorType
        if t == CompressorType.IDENTICAL:
            return d
        if t == CompressorType.LAZY_COMPRESSOR:
            return d if self.testp < self.P else 0
        if t in (CompressorType.RANDK_COMPRESSOR, CompressorType.TOPK_COMPRESSOR):
            return self.K
        if t == CompressorType.NATURAL_COMPRESSOR_FP32:
            return 9.0 / 32.0 * d
        if t == CompressorType.RANK_K_COMPRESSOR:
            # only the dyadic expansion is sent: K' (A + B), K' = min(K, min(A, B)) (compressors.py:348, 362)
            return min(self.K, self.A, self.B) * (self.A + self.B)
        return 1.0 + d * (1.0 + math.ceil(math.log2(self.s))) / 32.0

    def _account(self, d):
        self.last_input_advance = d
        self.last_need_to_send_advance = self._need_to_send(d)
        self.really_need_to_send_components += self.last_need_to_send_advance
        self.total_input_components += self.last_input_advance

    def compressVector(self, x):
        d = max(x.shape)
        if self.compressorType == CompressorType.IDENTICAL:
            out = x                                                     # alias, like the reference
        elif self._torch_norm():
            out = self._encode_gpu(x, pnorm_in=self.torchNorm(x))
        else:
            out = self._encode_gpu(x)
        self._account(d)
        return out

    def _torch_norm(self):
        mode = getattr(self, "norm_mode", "exact")
        if mode not in ("exact", "torch_cpu"):
            raise ValueError(f"norm_mode must be 'exact' or 'torch_cpu' (got {mode!r})")
        # standard dithering / QSGD (compressors.py:272) and natural dithering (303, whose output
        # y * sign * pnorm carries the norm's bits) both take torch.norm(x, p)
        if mode == "exact" or self.compressorType not in (CompressorType.STANDARD_DITHERING_FP32,
                                                          CompressorType.NATURAL_DITHERING_FP32):
            return False
        if self.p == 2:
            return True
        if self.p == math.inf:
            return False                       # max |x_j|: no rounding, every order gives it
        raise NotImplementedError(f"norm_mode='torch_cpu' restates torch's p=2 reduction only (p={self.p})")

    def torchNorm(self, x):
        """torch.norm(x, p=2) as the reference's CPU fp32 path computes it (compressors.py:272),
        bit for bit, on the GPU (flc_norm2_torch_cpu): a [1] fp32 device tensor."""
        if x.dtype != torch.float32:
            raise TypeError(f"flcodec encodes fp32 only (got {x.dtype})")
        dev = _gpu_device(x)
        xd = x.reshape(-1).to(device=dev).contiguous()
        out = torch.empty(1, dtype=torch.float32, device=dev)
        lib = _lib.load()
        d = xd.numel()
        # the chain's exact parallel form (flc_norm2_torch_cpu_ws: binade-segment maps, three
        # launches, ~0.1 ms at D = 25 M) — the same bits as the sequential chain
        ws = _lib.WORKSPACE.get(dev, lib.flc_norm2_torch_cpu_workspace_size(1, d))
        with torch.cuda.device(dev):
            rc = lib.flc_norm2_torch_cpu_ws(ctypes.c_void_p(xd.data_ptr()), d, 1, d, ctypes.c_void_p(out.data_ptr()),
                                            ctypes.c_void_p(ws.data_ptr()), ws.numel(), _lib.stream_ptr(dev))
        _lib.check(rc, "flc_norm2_torch_cpu_ws")
        return out

    def _pattern(self, dev, keep):
        """flc_pattern for this compressor's current pattern (compat mode) or device-RNG key."""
        t = self.compressorType
        pat = _lib.FlcPattern()
        if self.device_rng is not None:
            pat.client0 = int(self.device_rng[1])
        if t == CompressorType.LAZY_COMPRESSOR:
            u = torch.tensor([self.testp], dtype=torch.float64, device=dev)
            pat.d_lazy_u = u.data_ptr()
            keep.append(u)
        elif t == CompressorType.RANDK_COMPRESSOR and self.device_rng is None:
            if self.S.device != dev:
                self.S = self.S.to(device=dev)
            S = self.S.to(torch.int64).contiguous()
            pat.d_randk_idx = S.data_ptr()
            pat.idx_ld = S.numel()
            keep.append(S)
        elif t in (CompressorType.NATURAL_COMPRESSOR_FP32, CompressorType.STANDARD_DITHERING_FP32,
                   CompressorType.NATURAL_DITHERING_FP32) and self.device_rng is None:
            if self.testp.device != dev:
                self.testp = self.testp.to(device=dev, non_blocking=True)
            pat.d_uniforms = self.testp.data_ptr()
        return pat

    def _encode_gpu(self, x, pnorm_in=None, pnorm_out=None):
        if x.dtype != torch.float32:
            raise TypeError(f"flcodec encodes fp32 only (got {x.dtype})")
        dev = _gpu_device(x)
        host_in = not x.is_cuda
        xd = x.reshape(-1).to(device=dev).contiguous()
        d = xd.numel()
        lib = _lib.load()
        prm, keep = self.codec_params(dev)
        pat = self._pattern(dev, keep)
        out = torch.empty_like(xd)
        ws_bytes = lib.flc_encode_workspace_size(ctypes.byref(prm), d)
        ws = _lib.WORKSPACE.get(dev, ws_bytes)
        with torch.cuda.device(dev):
            rc = lib.flc_encode(ctypes.byref(prm), ctypes.byref(pat), ctypes.c_void_p(xd.data_ptr()), d,
                                ctypes.c_void_p(pnorm_in.data_ptr() if pnorm_in is not None else None),
                                ctypes.c_void_p(pnorm_out.data_ptr() if pnorm_out is not None else None),
                                ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(ws.data_ptr()), ws.numel(),
                                _lib.stream_ptr(dev))
        _lib.check(rc, "flc_encode")
        out = out.reshape(x.shape)
        return out.to("cpu") if host_in else out

    # -- wire format ------------------------------------------------------
    def _host_params(self):
        """flc_codec_params without device resources (sizes, formats, host-side checks)."""
        if self.compressorType in (CompressorType.STANDARD_DITHERING_FP32, CompressorType.NATURAL_DITHERING_FP32):
            prm = _lib.FlcCodecParams()
            prm.codec = int(self.compressorType)
            prm.s = int(self.s)
            return prm
        return self.codec_params(torch.device("cpu"))[0]

    def payloadBytes(self, d=None):
        """Bytes of one row's payload (flc_payload_bytes: 16-B header + body, 16-B padded)."""
        return int(_lib.load().flc_payload_bytes(ctypes.byref(self._host_params()), self._dim(d)))

    def validatePayload(self, payload, d=None):
        """Check a message received from a peer before it is decoded (flc_payload_validate, host
        only): its size, header and codes fit this codec and d.  ``payload``: bytes-like, a uint8
        numpy array or a host uint8 tensor.  Raises ValueError with the reason."""
        if torch.is_tensor(payload):
            if payload.dtype != torch.uint8 or payload.is_cuda:
                raise TypeError("validatePayload: a host uint8 tensor (or bytes) is expected")
            arr = payload.contiguous().numpy()
        else:
            arr = np.frombuffer(payload, dtype=np.uint8)
        lib = _lib.load()
        rc = lib.flc_payload_validate(ctypes.byref(self._host_params()), ctypes.c_void_p(arr.ctypes.data),
                                      int(arr.nbytes), self._dim(d))
        _lib.check(rc, "validatePayload")

    def _dim(self, d):
        if d is None:
            d = getattr(self, "D", None)
        if d is None:
            raise ValueError("this compressor has no D (identity): pass d")
        return int(d)

    def compressPayload(self, x, out=None):
        """The message this client would send: flc_pack of compressVector(x) (same pattern, same
        draws), as a uint8 device tensor of payloadBytes() bytes.  Statistics advance like
        compressVector."""
        if x.dtype != torch.float32:
            raise TypeError(f"flcodec encodes fp32 only (got {x.dtype})")
        dev = _gpu_device(x)
        xd = x.reshape(-1).to(device=dev).contiguous()
        d = xd.numel()
        lib = _lib.load()
        prm, keep = self.codec_params(dev)
        pat = self._pattern(dev, keep)
        nbytes = int(lib.flc_payload_bytes(ctypes.byref(prm), d))
        if out is None:
            out = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        elif out.numel() < nbytes or out.dtype != torch.uint8 or out.data_ptr() % 16:
            raise ValueError("compressPayload: out must be a 16-byte aligned uint8 tensor of payloadBytes()")
        ws_bytes = lib.flc_pack_workspace_size(ctypes.byref(prm), d)
        ws = _lib.WORKSPACE.get(dev, ws_bytes)
        with torch.cuda.device(dev):
            rc = lib.flc_pack(ctypes.byref(prm), ctypes.byref(pat), ctypes.c_void_p(xd.data_ptr()), d,
                              ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(ws.data_ptr()), ws.numel(),
                              _lib.stream_ptr(dev))
        _lib.check(rc, "flc_pack")
        self._account(d)
        return out

    def decompressPayload(self, payload, d=None):
        """Dense fp32 row of a payload (flc_unpack): compressVector's output, bit for bit."""
        dev = _gpu_device(payload)
        d = self._dim(d)
        lib = _lib.load()
        prm, keep = self.codec_params(dev)
        if payload.dtype != torch.uint8:
            raise TypeError(f"decompressPayload: payload must be uint8 (got {payload.dtype})")
        nbytes = int(lib.flc_payload_bytes(ctypes.byref(prm), d))
        if payload.numel() < nbytes:
            raise ValueError(f"decompressPayload: {payload.numel()} bytes, the payload of d={d} is {nbytes}")
        # a host message (off the network) crosses to the device first; the kernel reads HBM only
        payload = payload.reshape(-1)[:nbytes].to(device=dev)
        if not payload.is_contiguous() or payload.data_ptr() % 16:
            payload = payload.clone()
        out = torch.empty(d, dtype=torch.float32, device=dev)
        with torch.cuda.device(dev):
            rc = lib.flc_unpack(ctypes.byref(prm), ctypes.c_void_p(payload.data_ptr()), d,
                                ctypes.c_void_p(out.data_ptr()), _lib.stream_ptr(dev))
        _lib.check(rc, "flc_unpack")
        return out

    # -- shift codecs ----------------------------------------------------
    def compressShift(self, a, b, *, scale=1.0, base=None, out=None, alpha=None, shift=None, shift_out=None,
                      message=True, pnorm_out=None):
        """One fused pass of ``base + compressVector(a - b) * scale`` and ``shift + alpha * C(a - b)``.

        The torch expressions of the compressed algorithms' client step (DIANA algorithms.py:1383-1391,
        EF21 1506-1517, MARINA 537 / 691, FRECON 1104-1110, COFIG 1265-1269), fp32 op for op: the
        scalars are taken as fp32, like torch's tensor-scalar ops.  Returns ``(msg, shift_out)``
        (``msg`` None when ``message`` is False, ``shift_out`` None without ``alpha``).  ``out`` /
        ``shift_out`` may be any of the inputs (in-place update).  Updates the wire statistics
        like ``compressVector``.  Device tensors only (the client state lives on the GPU)."""
        for name, v in (("a", a), ("b", b), ("base", base), ("shift", shift), ("out", out),
                        ("shift_out", shift_out)):
            if v is not None and (v.dtype != torch.float32 or not v.is_cuda):
                raise TypeError(f"compressShift: {name} must be an fp32 device tensor")
        dev = _gpu_device(a)
        d = a.numel()
        if b.numel() != d or (base is not None and base.numel() != d) or (shift is not None and shift.numel() != d):
            raise ValueError("compressShift: a, b, base and shift must have the same number of elements")
        if alpha is not None and shift is None:
            raise ValueError("compressShift: alpha given without a shift tensor")
        keep = []

        def flat(v):
            if v is None:
                return None
            f = v.reshape(-1)
            if not f.is_contiguous():
                f = f.contiguous()
            keep.append(f)
            return f
        af, bf, basef, hf = flat(a), flat(b), flat(base), flat(shift)
        msg = None
        if message:
            msg = out if out is not None else torch.empty_like(af)
            if not msg.is_contiguous():
                raise ValueError("compressShift: out must be contiguous")
        hout = None
        if alpha is not None:
            hout = shift_out if shift_out is not None else torch.empty_like(hf)
            if not hout.is_contiguous():
                raise ValueError("compressShift: shift_out must be contiguous")
        if msg is None and hout is None:
            raise ValueError("compressShift: nothing to compute (message=False and no alpha)")
        lib = _lib.load()
        prm, k2 = self.codec_params(dev)
        keep.extend(k2)
        pat = self._pattern(dev, keep)
        ws_bytes = lib.flc_encode_shift_workspace_size(ctypes.byref(prm), d)
        ws = _lib.WORKSPACE.get(dev, ws_bytes)
        vp = ctypes.c_void_p

        def ptr(v):
            return vp(v.data_ptr() if v is not None else None)
        with torch.cuda.device(dev):
            rc = lib.flc_encode_shift(ctypes.byref(prm), ctypes.byref(pat), ptr(af), ptr(bf), d,
                                      ctypes.c_float(float(np.float32(scale))), ptr(basef), ptr(msg),
                                      ctypes.c_float(float(np.float32(alpha if alpha is not None else 0.0))),
                                      ptr(hf if hout is not None else None), ptr(hout), ptr(pnorm_out),
                                      vp(ws.data_ptr()), ws.numel(), _lib.stream_ptr(dev))
        _lib.check(rc, "flc_encode_shift")
        self._account(d)
        if msg is not None:
            msg = msg.view(a.shape)
        if hout is not None:
            hout = hout.view(shift.shape)
        return msg, hout


def initCompressor(compressorCmdLine, D):
    """Spec grammar of compressors.py:435-494: name[:arg[:arg]], K as count or percent."""
    params = compressorCmdLine.split(":")
    name = params[0]
    c = Compressor()

    def count_or_percent(arg):
        if arg.find("%") == -1:
            return math.ceil(float(arg))
        return math.ceil(float(arg[0:-1]) / 100.0 * D)

    def pnorm_arg():
        if len(params) == 3:
            return math.inf if params[2].lower() == "inf" else int(params[2])
        return math.inf

    if name == "ident":
        c.makeIdenticalCompressor()
    elif name == "randk":
        c.makeRandKCompressor(D, count_or_percent(params[1]))
    elif name == "bernulli":
        c.makeLazyCompressor(float(params[1]))
    elif name == "natural":
        c.makeNaturalCompressorFP32(D)
    elif name == "qsgd":
        c.makeQSGD_FP32(D, int(params[1]))
    elif name == "nat.dithering":
        c.makeNaturalDitheringFP32(D, int(params[1]), pnorm_arg())
    elif name == "std.dithering":
        c.makeStandardDitheringFP32(D, int(params[1]), pnorm_arg())
    elif name == "topk":
        c.makeTopKCompressor(D, count_or_percent(params[1]))
    elif name == "rank_k":
        c.makeRankKCompressor(D, count_or_percent(params[1]))
    elif name == "terngrad":
        c.makeTernGrad(D)
    else:
        raise AssertionError("Unknown compressor format")
    return c
