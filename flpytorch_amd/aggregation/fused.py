"""Fused uplink of one round: encode every client row with its codec and reduce, one call.

    out = (sum_i w_i * C_i(g_i)) / sum(w)        (flc_encode_reduce)

``C_i`` is the compressor of client i (``compressors.py:218-371``) under its own pattern; the sum
runs in client order with fp32 rounding per operation, i.e. bit-identical to encoding each row
with ``compressVector`` and reducing the dense outputs sequentially (the reference's
``serverGradient`` order, algorithms.py:1753-1768) — without materialising the N dense outputs.

Pattern sources
  * compat  — the reference's numpy stream: RandK index sets [N, K] int64 and dithering /
              natural uniforms [N, D] float64 drawn on the host (``stream_choice`` /
              ``stream_rand``) and uploaded; lazy draws [N] float64.
  * device  — counter-based draws keyed by (seed, client id, element) generated inside the
              kernels: no host work, no uniform bytes (the benchmark mode).
"""
import ctypes

import torch

from .. import _lib
from .compressors import Compressor, CompressorType


def _device(device):
    """torch.device with its index resolved (``'cuda'`` -> the current device), so that it compares
    equal to a stream's device."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if dev.type == "cuda" and dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    return dev


def select_row_flags(comp: Compressor, n, d, device=None):
    """Path report of the last TopK call on the current stream's workspace (flc_select_row_flags): a
    [n] int64 tensor of row state bits — 1 overflow, 2 short list, 4 ties cut on the fast path,
    8 exact path, 16 a lone row selected in registers (compressVector, D <= 16.7 M).  Call it right after the UplinkReducer / compressVector call, with its n and d
    (compressVector: n = 1).  Tests use it to assert which path ran."""
    dev = _device(device)
    lib = _lib.load()
    prm, _ = comp.codec_params(dev)
    ws_bytes = lib.flc_encode_reduce_workspace_size(ctypes.byref(prm), n, d)
    ws = _lib.WORKSPACE.get(dev, ws_bytes)
    flags = torch.zeros(n, dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        rc = lib.flc_select_row_flags(ctypes.byref(prm), n, d, ctypes.c_void_p(ws.data_ptr()), ws.numel(),
                                      ctypes.c_void_p(flags.data_ptr()), _lib.stream_ptr(dev))
    _lib.check(rc, "flc_select_row_flags")
    return flags.cpu().to(torch.int64)


class UplinkReducer:
    """Holds the codec constants + workspace for repeated fused encode+reduce calls."""

    def __init__(self, compressor: Compressor, device=None, seed=None):
        _lib.require_gpu()
        self.comp = compressor
        self.device = _device(device)
        self.seed = seed

    def params(self):
        prm, keep = self.comp.codec_params(self.device)
        if self.seed is not None:
            prm.seed = int(self.seed) & 0xFFFFFFFFFFFFFFFF
        return prm, keep

    def workspace_bytes(self, n, d):
        prm, _ = self.params()
        return _lib.load().flc_encode_reduce_workspace_size(ctypes.byref(prm), n, d)

    def randk_counts(self, n, d, client0=0, out=None):
        """The device sampler's chunk counts [ceil(d / 4096), n] (uint32 as int32) of clients
        client0.. on the current stream (flc_device_randk_counts) — pure compute, no row is read;
        hand them to __call__(randk_counts=...) to take that work out of the call."""
        lib = _lib.load()
        dev = self.device
        if self.seed is None:
            raise ValueError("device-RNG counts need a seed")
        C = (d + 4095) // 4096
        if out is None:
            out = torch.empty((C, n), dtype=torch.int32, device=dev)
        wsb = lib.flc_device_randk_counts_workspace_size(n, d)
        if getattr(self, "_cnt_ws", None) is None or self._cnt_ws.numel() < wsb:
            self._cnt_ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        with torch.cuda.device(dev):
            rc = lib.flc_device_randk_counts(int(self.seed) & 0xFFFFFFFFFFFFFFFF, int(client0), n, d, self.comp.K,
                                             ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(self._cnt_ws.data_ptr()),
                                             self._cnt_ws.numel(), _lib.stream_ptr(dev))
        _lib.check(rc, "flc_device_randk_counts")
        return out

    def __call__(self, rows, out=None, weights=None, client0=0, randk_idx=None, uniforms=None, lazy_u=None,
                 pnorms_out=None, stream=None, divisor=None, randk_counts=None):
        """rows: [N, D] fp32 device tensor (row stride % 4 == 0 for the vector path) or a list of
        [D] device tensors.  Compat patterns: randk_idx [N, K] int64, uniforms [N, D] float64,
        lazy_u [N] float64 (device).  Without them (and with ``seed`` set) draws are on device.
        ``divisor`` overrides the fp32 divisor sum(w) (e.g. 1.0 for a partial sum across GPUs).
        ``stream``: every allocation, copy and the launch go to that stream (torch's stream
        semantics: the caller orders it after the producers of ``rows`` and the patterns).
        ``randk_counts``: RandK device mode, the chunk counts from ``randk_counts(n, d, client0)``."""
        if stream is not None:
            if stream.device != self.device:
                raise ValueError(f"stream is on {stream.device}, the reducer runs on {self.device}")
            with torch.cuda.stream(stream):
                return self._run(rows, out, weights, client0, randk_idx, uniforms, lazy_u, pnorms_out, divisor,
                                 randk_counts)
        return self._run(rows, out, weights, client0, randk_idx, uniforms, lazy_u, pnorms_out, divisor, randk_counts)

    def _run(self, rows, out, weights, client0, randk_idx, uniforms, lazy_u, pnorms_out, divisor, randk_counts=None):
        """The call on the current stream (allocations, uploads and the launch all on it)."""
        lib = _lib.load()
        dev = self.device
        if self.comp._torch_norm():
            raise NotImplementedError("UplinkReducer folds with exactly rounded norms; norm_mode='torch_cpu' "
                                      "(the reference's CPU norm bits) is served by compressVector")
        prm, keep = self.params()
        pat = _lib.FlcPattern()
        pat.client0 = int(client0)
        if torch.is_tensor(rows) and rows.dim() == 2:
            n, d = rows.shape
            base, ld, ptrs = rows.data_ptr(), rows.stride(0), None
            if rows.stride(1) != 1:
                raise ValueError("rows must be row-contiguous")
        else:
            n = len(rows)
            d = rows[0].numel() if n else 0
            # the pointer-array entry reads rows with 16-byte vector loads: keep them aligned
            rows = [r if (r.is_contiguous() and r.data_ptr() % 16 == 0) else r.contiguous().clone() for r in rows]
            keep.extend(rows)
            # pinned staging + async copy: no host wait on the work already queued on the stream
            host_pt = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64).pin_memory()
            pt = host_pt.to(dev, non_blocking=True)
            keep.append(pt)
            base, ld, ptrs = None, 0, pt.data_ptr()
        if out is None:
            out = torch.empty(d, dtype=torch.float32, device=dev)
        if n == 0:
            return out.zero_()                                   # no clients (algorithms.py:2117-2118)
        t = self.comp.compressorType
        if t == CompressorType.RANDK_COMPRESSOR and randk_idx is not None:
            pat.d_randk_idx = randk_idx.data_ptr()
            pat.idx_ld = randk_idx.stride(0)
        if randk_counts is not None and t == CompressorType.RANDK_COMPRESSOR and randk_idx is None:
            if tuple(randk_counts.shape) != ((d + 4095) // 4096, n) or not randk_counts.is_cuda:
                raise ValueError("randk_counts must be a [ceil(d / 4096), n] device tensor")
            pat.d_randk_counts = randk_counts.data_ptr()
        if uniforms is not None:
            pat.d_uniforms = uniforms.data_ptr()
            pat.uniforms_ld = uniforms.stride(0)
        if t == CompressorType.LAZY_COMPRESSOR:
            if lazy_u is None:
                raise ValueError("lazy codec needs lazy_u [N] draws")
            pat.d_lazy_u = lazy_u.data_ptr()
        needs_seed = (t in (CompressorType.RANDK_COMPRESSOR,) and randk_idx is None) or \
                     (t in (CompressorType.NATURAL_COMPRESSOR_FP32, CompressorType.STANDARD_DITHERING_FP32)
                      and uniforms is None)
        if needs_seed and self.seed is None:
            raise ValueError("no compat pattern given and no device-RNG seed set")
        w_ptr, total = None, float(n)
        if weights is not None:
            weights = [float(w) for w in weights]
            total = weights[0]
            for w in weights[1:]:
                total += w
            wt = torch.tensor(weights, dtype=torch.float32, device=dev)
            keep.append(wt)
            w_ptr = wt.data_ptr()
        if divisor is not None:
            total = float(divisor)
        ws_bytes = lib.flc_encode_reduce_workspace_size(ctypes.byref(prm), n, d)
        ws = _lib.WORKSPACE.get(dev, ws_bytes)
        st = _lib.stream_ptr(dev)
        with torch.cuda.device(dev):
            rc = lib.flc_encode_reduce(ctypes.byref(prm), ctypes.byref(pat), ctypes.c_void_p(base), ld,
                                       ctypes.c_void_p(ptrs), n, d, ctypes.c_void_p(w_ptr), ctypes.c_float(total),
                                       ctypes.c_void_p(pnorms_out.data_ptr() if pnorms_out is not None else None),
                                       ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(ws.data_ptr()), ws.numel(), st)
        _lib.check(rc, "flc_encode_reduce")
        return out


class PayloadReducer:
    """Server side of the wire format: out = (sum_i w_i * decode(payload_i)) / sum(w), folded in
    client order straight from the messages (flc_unpack_reduce) — the same bits as
    flc_encode_reduce of the rows the payloads were packed from."""

    def __init__(self, compressor: Compressor, device=None):
        _lib.require_gpu()
        self.comp = compressor
        self.device = _device(device)

    def __call__(self, payloads, d=None, out=None, weights=None, divisor=None):
        """payloads: [N, ld] uint8 device tensor (rows 16-byte aligned, ld % 16 == 0) or a list of
        uint8 device tensors."""
        lib = _lib.load()
        dev = self.device
        d = self.comp._dim(d)
        prm, keep = self.comp.codec_params(dev)
        if torch.is_tensor(payloads) and payloads.dim() == 2:
            n, ld = payloads.shape
            if payloads.stride(1) != 1 or payloads.stride(0) % 16 or payloads.data_ptr() % 16:
                raise ValueError("payload rows must be contiguous and 16-byte aligned")
            base, ldb, ptrs = payloads.data_ptr(), payloads.stride(0), None
        else:
            n = len(payloads)
            for p in payloads:
                if p.data_ptr() % 16:
                    raise ValueError("payloads must be 16-byte aligned")
            host_pt = torch.tensor([p.data_ptr() for p in payloads], dtype=torch.int64).pin_memory()
            pt = host_pt.to(dev, non_blocking=True)
            keep.extend(payloads)
            keep.append(pt)
            base, ldb, ptrs = None, 0, pt.data_ptr()
        if out is None:
            out = torch.empty(d, dtype=torch.float32, device=dev)
        w_ptr, total = None, float(n)
        if weights is not None:
            weights = [float(w) for w in weights]
            total = weights[0]
            for w in weights[1:]:
                total += w
            wt = torch.tensor(weights, dtype=torch.float32, device=dev)
            keep.append(wt)
            w_ptr = wt.data_ptr()
        if divisor is not None:
            total = float(divisor)
        ws_bytes = lib.flc_unpack_reduce_workspace_size(ctypes.byref(prm), n, d)
        ws = _lib.WORKSPACE.get(dev, ws_bytes)
        with torch.cuda.device(dev):
            rc = lib.flc_unpack_reduce(ctypes.byref(prm), ctypes.c_void_p(base), ldb, ctypes.c_void_p(ptrs), n, d,
                                       ctypes.c_void_p(w_ptr), ctypes.c_float(total), ctypes.c_void_p(out.data_ptr()),
                                       ctypes.c_void_p(ws.data_ptr()), ws.numel(), _lib.stream_ptr(dev))
        _lib.check(rc, "flc_unpack_reduce")
        return out
