"""Clients sharded across GPUs: one process per GPU, a [D] partial per GPU, one collective.

The reference's only multi-GPU scheme is worker threads round-robin over a `--gpu` device list
with a per-client `.to(device)` copy to the master inside every serverGradient
(fl_pytorch/utils/thread_pool.py:59; algorithms.py:1756, 1763).  Here each rank owns a
contiguous block of the round's clients, encodes + reduces them locally in client order
(flc_encode_reduce with fp32 divisor 1.0, i.e. the exact partial sum) and the partials meet in a
single collective over RCCL/xGMI (torch.distributed backend "nccl" on ROCm; "gloo" in the CPU
tests).  Then every rank divides by the global weight.

Two combine modes:
  * "allreduce" — one all-reduce(SUM) of D floats (bandwidth-optimal; RCCL's sum order);
  * "ordered"   — all-gather of the partials and a fixed rank-order fold: the result depends
                  only on the client->rank blocks, bit-reproducible run to run.
"""
import torch
import torch.distributed as dist


def client_block(n_clients, world, rank):
    """Contiguous, balanced block [lo, hi) of client positions owned by `rank`."""
    base, extra = divmod(n_clients, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


class ShardedUplink:
    """Round-level uplink over a process group.

    encode_partial(rows, client0, out) must write sum_i w_i C_i(rows_i) (no division) into `out`
    — the product passes an UplinkReducer with divisor=1.0; tests may pass an oracle callable.
    """

    def __init__(self, encode_partial, group=None, mode="allreduce"):
        if mode not in ("allreduce", "ordered"):
            raise ValueError(mode)
        self.encode_partial = encode_partial
        self.group = group
        self.mode = mode

    def __call__(self, rows, client0, total_weight, out=None):
        world = dist.get_world_size(self.group)
        d = rows.shape[1] if torch.is_tensor(rows) else rows[0].numel()
        dev = rows.device if torch.is_tensor(rows) else rows[0].device
        if out is None:
            out = torch.empty(d, dtype=torch.float32, device=dev)
        n_local = rows.shape[0] if torch.is_tensor(rows) else len(rows)
        if n_local:
            self.encode_partial(rows, client0, out)
        else:
            out.zero_()
        if world > 1:
            if self.mode == "allreduce":
                dist.all_reduce(out, group=self.group)
            else:
                parts = [torch.empty_like(out) for _ in range(world)]
                dist.all_gather(parts, out, group=self.group)
                out.copy_(parts[0])
                for p in parts[1:]:
                    out.add_(p)
        # a device-tensor divisor: torch turns a Python-scalar division on the GPU into a multiply
        # by the reciprocal; the fold's contract (and the reference CPU path) is a true fp32 division
        out.div_(torch.tensor(float(total_weight), dtype=torch.float32, device=out.device))
        return out


def product_partial(reducer):
    """encode_partial backed by the HIP kernels (flc_encode_reduce, fp32 divisor 1.0)."""

    def run(rows, client0, out):
        reducer(rows, out=out, client0=client0, divisor=1.0)
    return run


# ---------------------------------------------------------------------------------------------
# The C-ABI combine (flc_combine_partials) on a caller-owned RCCL communicator: the path a non-torch
# host (the C ABI's own callers) takes; torch.distributed's communicator stays private to torch.
# ---------------------------------------------------------------------------------------------
class RcclComm:
    """A caller-owned RCCL communicator over the ranks of a torch.distributed group (any backend:
    the 128-byte unique id travels through it), one GPU per rank."""

    def __init__(self, group=None):
        import ctypes
        import os
        # one node: RCCL's bootstrap on the loopback interface unless the caller chose one
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        self._ct = ctypes
        self.lib = ctypes.CDLL("librccl.so")

        class UniqueId(ctypes.Structure):
            _fields_ = [("internal", ctypes.c_char * 128)]
        self._uid_t = UniqueId
        self.lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(UniqueId)]
        self.lib.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, UniqueId, ctypes.c_int]
        self.lib.ncclCommDestroy.argtypes = [ctypes.c_void_p]
        rank = dist.get_rank(group)
        world = dist.get_world_size(group)
        uid = UniqueId()
        if rank == 0:
            if self.lib.ncclGetUniqueId(ctypes.byref(uid)) != 0:
                raise RuntimeError("ncclGetUniqueId failed")
        # the raw 128 bytes (a c_char array field reads back only up to its first NUL)
        box = [ctypes.string_at(ctypes.addressof(uid), 128) if rank == 0 else None]
        dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        ctypes.memmove(ctypes.addressof(uid), box[0], 128)
        self.ptr = ctypes.c_void_p()
        rc = self.lib.ncclCommInitRank(ctypes.byref(self.ptr), world, uid, rank)
        if rc != 0:
            self.lib.ncclGetErrorString.restype = ctypes.c_char_p
            raise RuntimeError(f"ncclCommInitRank failed: {rc} {self.lib.ncclGetErrorString(rc).decode()}")
        self.world = world

    def destroy(self):
        if self.ptr:
            self.lib.ncclCommDestroy(self.ptr)
            self.ptr = self._ct.c_void_p()


def combine_partials(comm, partial, total_weight, ordered=False):
    """In place: partial <- (sum over ranks of partial) / total_weight through flc_combine_partials
    (FLC_COMBINE_ORDERED: fixed rank-order fold, bit-reproducible)."""
    import ctypes
    from . import _lib
    lib = _lib.load()
    mode = 1 if ordered else 0
    d = partial.numel()
    ws_bytes = lib.flc_combine_workspace_size(comm.ptr, d, mode)
    ws = _lib.WORKSPACE.get(partial.device, ws_bytes) if ws_bytes else None
    with torch.cuda.device(partial.device):
        rc = lib.flc_combine_partials(comm.ptr, ctypes.c_void_p(partial.data_ptr()), d, ctypes.c_float(float(total_weight)),
                                      mode, ctypes.c_void_p(ws.data_ptr() if ws is not None else None),
                                      ws.numel() if ws is not None else 0, _lib.stream_ptr(partial.device))
    _lib.check(rc, "flc_combine_partials")
    return partial
