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
  * "ordered"   — G-invariant: the round's clients fall into N_BLOCKS = 8 fixed
                  contiguous blocks, rank r of G owns blocks r*8/G .. (r+1)*8/G - 1 and computes
                  one exact partial per block; an all-to-all hands rank r column slice r of every
                  block partial, the 8 slices are folded in block order
                  (((p_0 + p_1) + p_2) + ...) / w_total, and an all-gather assembles the result.
                  The bits depend only on the 8 blocks, never on G (1, 2, 4 or 8 GPUs give the
                  same result) and the traffic is a ring all-reduce's: 2 (G-1)/G x 4 D bytes
                  per rank when every rank owns one block.
"""
import torch
import torch.distributed as dist


def client_block(n_clients, world, rank):
    """Contiguous, balanced block [lo, hi) of client positions owned by `rank`."""
    base, extra = divmod(n_clients, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


N_BLOCKS = 8


def rank_blocks(world, rank, n_blocks=N_BLOCKS):
    """The fixed client blocks rank `rank` of `world` owns in "ordered" mode (contiguous)."""
    if world < 1 or n_blocks % world:
        raise ValueError(f"ordered mode needs the {n_blocks} client blocks split evenly over {world} ranks")
    per = n_blocks // world
    return range(rank * per, (rank + 1) * per)


def rank_clients(n_clients, world, rank, n_blocks=N_BLOCKS):
    """[lo, hi) of the clients rank `rank` owns in "ordered" mode: the union of its blocks."""
    bl = rank_blocks(world, rank, n_blocks)
    return client_block(n_clients, n_blocks, bl.start)[0], client_block(n_clients, n_blocks, bl.stop - 1)[1]


def combine_blocks(parts, total_weight, fold, group=None):
    """parts: [nb_local, D] exact block partials of this rank's blocks (block order).  Returns the
    [D] result (sum over ALL blocks in block order) / total_weight on every rank.

    fold(stack [B, S], total) -> [S] must compute (((s_0 + s_1) + s_2) + ...) / total in fp32 —
    product_fold() on the GPU, a sequential torch fold in the CPU tests."""
    nb, d = parts.shape
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1:
        return fold(parts, total_weight)
    # column slice per rank, padded to a 16-byte multiple (aligned collective buffers)
    s = -(-d // world)
    s = (s + 3) // 4 * 4
    send = parts.new_zeros((world, nb, s))
    padded = parts.new_zeros((nb, world * s))
    padded[:, :d] = parts
    send.copy_(padded.view(nb, world, s).transpose(0, 1))
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    # recv[q] = rank q's blocks (contiguous, rank order) of my slice: [8 blocks, s] in block order
    mine = fold(recv.view(world * nb, s), total_weight).contiguous()
    gathered = parts.new_empty(world * s)
    dist.all_gather_into_tensor(gathered, mine, group=group)
    return gathered[:d]


class ShardedUplink:
    """Round-level uplink over a process group.

    encode_partial(rows, client0, out) must write sum_i w_i C_i(rows_i) (no division) into `out`
    — the product passes an UplinkReducer with divisor=1.0; tests may pass an oracle callable.
    "ordered" mode also needs `fold` (see combine_blocks) and the round's client count.
    """

    def __init__(self, encode_partial, group=None, mode="allreduce", fold=None, n_blocks=N_BLOCKS):
        if mode not in ("allreduce", "ordered"):
            raise ValueError(mode)
        if mode == "ordered" and fold is None:
            raise ValueError("ordered mode needs a block fold (product_fold() on the GPU)")
        self.encode_partial = encode_partial
        self.group = group
        self.mode = mode
        self.fold = fold
        self.n_blocks = n_blocks
        self._parts = None

    def __call__(self, rows, client0, total_weight, out=None, n_clients=None, d=None, device=None):
        """allreduce: `rows` are this rank's clients, the first one is client `client0`.
        ordered: `rows` are this rank's clients rank_clients(n_clients, G, rank) (client0 is their
        first), or a callable rows(lo, hi) returning the rows of clients [lo, hi) (a resident shard
        replayed for each block; then pass d and device)."""
        world = dist.get_world_size(self.group) if dist.is_initialized() else 1
        if callable(rows):
            if d is None or device is None:
                raise ValueError("rows(lo, hi) needs d and device")
            dev = torch.device(device)
        else:
            d = rows.shape[1] if torch.is_tensor(rows) else rows[0].numel()
            dev = rows.device if torch.is_tensor(rows) else rows[0].device
        if self.mode == "ordered":
            res = self._ordered(rows, client0, total_weight, n_clients, d, dev, world)
            if out is None:
                return res
            return out.copy_(res)
        if out is None:
            out = torch.empty(d, dtype=torch.float32, device=dev)
        n_local = rows.shape[0] if torch.is_tensor(rows) else len(rows)
        if n_local:
            self.encode_partial(rows, client0, out)
        else:
            out.zero_()
        if world > 1:
            dist.all_reduce(out, group=self.group)
        # a device-tensor divisor: torch turns a Python-scalar division on the GPU into a multiply
        # by the reciprocal; the fold's contract (and the reference CPU path) is a true fp32 division
        out.div_(torch.tensor(float(total_weight), dtype=torch.float32, device=out.device))
        return out

    def _ordered(self, rows, client0, total_weight, n_clients, d, dev, world):
        if n_clients is None:
            raise ValueError("ordered mode needs n_clients (the round's client count)")
        rank = dist.get_rank(self.group) if world > 1 else 0
        lo, hi = rank_clients(n_clients, world, rank, self.n_blocks)
        blocks = rank_blocks(world, rank, self.n_blocks)
        if not callable(rows):
            n_local = rows.shape[0] if torch.is_tensor(rows) else len(rows)
            if client0 != lo or n_local != hi - lo:
                raise ValueError(f"rank {rank} owns clients [{lo}, {hi}) in ordered mode, got {n_local} from {client0}")
        if self._parts is None or self._parts.shape != (len(blocks), d) or self._parts.device != dev:
            self._parts = torch.empty((len(blocks), d), dtype=torch.float32, device=dev)
        for i, b in enumerate(blocks):
            b_lo, b_hi = client_block(n_clients, self.n_blocks, b)
            if b_hi == b_lo:
                # an empty block's partial is the additive identity -0: adding it keeps a column
                # that is -0 in every real block at -0, as the sequential fold does
                self._parts[i].fill_(-0.0)
            elif callable(rows):
                self.encode_partial(rows(b_lo, b_hi), b_lo, self._parts[i])
            else:
                self.encode_partial(rows[b_lo - lo:b_hi - lo], b_lo, self._parts[i])
        return combine_blocks(self._parts, total_weight, self.fold, self.group)


def product_partial(reducer):
    """encode_partial backed by the HIP kernels (flc_encode_reduce, fp32 divisor 1.0)."""

    def run(rows, client0, out):
        reducer(rows, out=out, client0=client0, divisor=1.0)
    return run


def product_fold():
    """The block fold on the GPU: flc_reduce_matrix (plain mode) over the [B, S] block slices with
    the global weight as the fp32 divisor — the sequential block-order sum, one pass."""
    from .aggregation.reduce import reduce_rows

    def fold(stack, total):
        return reduce_rows(stack[0], stack, relative=False, divisor=float(total))
    return fold


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


def combine_blocks_rccl(comm, parts, total_weight, out=None):
    """flc_combine_blocks: this rank's [nb_local, D] block partials -> the G-invariant [D] result
    (sum over all blocks in block order) / total_weight, on every rank."""
    import ctypes
    from . import _lib
    lib = _lib.load()
    nb, d = parts.shape
    if out is None:
        out = torch.empty(d, dtype=torch.float32, device=parts.device)
    ws_bytes = lib.flc_combine_blocks_workspace_size(comm.ptr, nb, d)
    ws = _lib.WORKSPACE.get(parts.device, ws_bytes) if ws_bytes else None
    with torch.cuda.device(parts.device):
        rc = lib.flc_combine_blocks(comm.ptr, ctypes.c_void_p(parts.data_ptr()), parts.stride(0), nb, d,
                                    ctypes.c_float(float(total_weight)), ctypes.c_void_p(out.data_ptr()),
                                    ctypes.c_void_p(ws.data_ptr() if ws is not None else None),
                                    ws.numel() if ws is not None else 0, _lib.stream_ptr(parts.device))
    _lib.check(rc, "flc_combine_blocks")
    return out
