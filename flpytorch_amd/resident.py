"""The resident client-update matrix: N client rows of D fp32 in one physically contiguous HBM
range (flc_rows_alloc, hipDeviceMallocContiguous) wrapped as a torch tensor.

Why: the uplink kernels stream every row once, at the HBM rate, and a default allocation of tens of
GB is stitched from physical fragments: some of its 6.4 GB blocks read at 5.6 TB/s beside 6.2 TB/s
ones, with 5-20 % more address-translation misses and fewer reads outstanding at the memory side
(profiles/r06/regions_pmc.jsonl) — which blocks are slow changes with every allocation.  Physically
contiguous memory is mapped with the largest page fragments: C4's 512 x 25 M shard read in 8.04
instead of 8.48 ms and its encode+reduce step took 9.09 instead of 9.57 ms, in one process with the
same bits (profiles/r06/contig.jsonl).  The reference keeps its N client tensors wherever torch
puts them (model_funcs.py:367-386); a simulator built on this package allocates the round's client
matrix once here and lets the clients' updates land in its rows.
"""
import ctypes
import warnings

import torch

from . import _lib


class _Rows:
    """Owner of one flc_rows_alloc range; torch keeps it alive as long as the tensor's storage."""

    def __init__(self, ptr, shape, dtype, device):
        self.ptr = ptr
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": {torch.float32: "<f4", torch.uint8: "|u1",
                                                                          torch.float64: "<f8"}[dtype],
                                         "data": (ptr, False), "version": 3, "strides": None}
        self._device = device

    def __del__(self):
        try:
            with torch.cuda.device(self._device):
                torch.cuda.synchronize(self._device)          # no kernel may still read the range
                _lib.load().flc_rows_free(ctypes.c_void_p(self.ptr))
        except Exception:  # noqa: BLE001 — interpreter shutdown: the process frees the device anyway
            pass


def resident_rows(n, d, dtype=torch.float32, device=None, contiguous=True):
    """An [n, d] tensor in one physically contiguous HBM range (contiguous=True, falling back to
    an ordinary device allocation with a warning when no contiguous range that large is free);
    returns (tensor, "contiguous" | "default")."""
    _lib.require_gpu()
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    nbytes = int(n) * int(d) * torch.tensor([], dtype=dtype).element_size()
    if contiguous and nbytes:
        lib = _lib.load()
        p = ctypes.c_void_p()
        with torch.cuda.device(dev):
            rc = lib.flc_rows_alloc(nbytes, 1, ctypes.byref(p))
        if rc == 0 and p.value:
            owner = _Rows(p.value, (n, d), dtype, dev)
            return torch.as_tensor(owner, device=dev), "contiguous"
        warnings.warn(f"resident_rows: no physically contiguous {nbytes / 1e9:.1f} GB range "
                      f"({_lib.load().flc_last_error_string().decode()}); default allocation")
    return torch.empty((n, d), dtype=dtype, device=dev), "default"
