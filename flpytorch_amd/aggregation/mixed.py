"""Mixed per-client codec uplink (BASELINE config C5; SURVEY §8d "C5").

The reference runs one client codec per experiment (H["client_compressor"], algorithms.py:2003;
its ProbabilisticSwitchingCompressor, compressors.py:395-432, is never constructed), so a mixed
round has no reference output: parity is per client, per constituent codec, and the
combination order is this module's own, stated here:

    client i (global id) uses codec g = i mod G;  group g's partial P_g = sum over its clients,
    in client order, of w_i C_g(row_i)  (flc_encode_reduce, divisor 1.0);
    out = (((P_0 + P_1) + P_2) + ...) / w_total           (fp32, left to right)

Device-RNG keys: group g draws with seed_g = seed + g * 0x9E3779B97F4A7C15 (mod 2^64) and client
number i // G, so every (codec, client) pair has its own stream.

Multi-GPU: with a process group, each group's [D] partial is all-reduced (RCCL over xGMI) as soon
as it is encoded, asynchronously, so the collective of group g overlaps the encode of group g+1
(the sum is linear: allreduce(sum_g P_g) = sum_g allreduce(P_g)).

RandK groups (HIP path, device draws): their chunk counts (k_randk_counts — the device sampler,
pure compute, no HBM traffic) are computed on a side stream at the start of the call, under the
other groups' streaming filters, and the RandK groups are encoded last from those counts.  Only
the counts overlap: the RandK fold's gathers beside a filter measured 20x slower.  The partials
land in separate buffers and are combined in group order, so the bits do not depend on this.
"""
import torch

import torch.distributed  # noqa: F401  (get_world_size / all_reduce when a group is given)

from .compressors import initCompressor
from .fused import UplinkReducer

_GOLDEN = 0x9E3779B97F4A7C15


class MixedUplink:
    def __init__(self, specs, D, seed, device=None, encode_partial=None):
        """encode_partial(g, rows_g, client_number0, out) writes group g's partial sum into out;
        default: the HIP kernels (flc_encode_reduce, device-RNG, fp32 divisor 1.0).  Tests pass
        an oracle callable (CPU tensors) to exercise the combine and the collectives."""
        self.specs = list(specs)
        self.G = len(self.specs)
        self.D = D
        self.seeds = [(int(seed) + g * _GOLDEN) & 0xFFFFFFFFFFFFFFFF for g in range(self.G)]
        if encode_partial is None:
            reducers = [UplinkReducer(initCompressor(sp, D), device=device, seed=sd)
                        for sp, sd in zip(self.specs, self.seeds)]
            self.device = reducers[0].device

            def encode_partial(g, rows_g, c0, out, counts=None):
                reducers[g](rows_g, out=out, client0=c0, divisor=1.0, randk_counts=counts)

            def counts_of(g, n_g, c0, out=None):
                return reducers[g].randk_counts(n_g, D, c0, out=out)
            self.counts_of = counts_of
            self.counts_groups = [g for g, sp in enumerate(self.specs) if sp.split(":")[0] == "randk"]
        else:
            self.device = torch.device(device) if device is not None else torch.device("cpu")
            self.counts_groups = []
        self.encode_partial = encode_partial
        self._parts = None
        self._side = None
        self._counts = {}

    def groups(self, client0, n):
        """Positions (0..n-1) of the clients client0..client0+n-1 in each codec group, and the client
        number (i // G) of each group's first member.  client0 must be a multiple of G."""
        if client0 % self.G:
            raise ValueError(f"client0={client0} must be a multiple of the codec count {self.G}")
        return [(list(range(g, n, self.G)), client0 // self.G) for g in range(self.G)]

    def partials(self, rows, client0=0, group=None):
        """The G partial sums [G, D] (each all-reduced over `group` when given; returns the pending
        collective handles too)."""
        n = rows.shape[0] if torch.is_tensor(rows) else len(rows)
        if self._parts is None or self._parts.shape[1] != self.D:
            self._parts = torch.empty((self.G, self.D), dtype=torch.float32, device=self.device)
        parts = self._parts
        handles = []
        grouped = self.groups(client0, n)
        early = [g for g in self.counts_groups if grouped[g][0]]
        counts = {}
        if early and len(early) < self.G:
            if self._side is None:
                self._side = torch.cuda.Stream(device=self.device)
            main = torch.cuda.current_stream(self.device)
            self._side.wait_stream(main)
            with torch.cuda.stream(self._side):
                for g in early:
                    pos, c0 = grouped[g]
                    buf = self._counts.get(g)
                    if buf is None or buf.shape[1] != len(pos):
                        buf = self._counts[g] = None
                    counts[g] = self._counts[g] = self.counts_of(g, len(pos), c0, out=buf)
            self._counts_ready = torch.cuda.Event()
            self._counts_ready.record(self._side)
        else:
            early = []

        def run(g):
            pos, c0 = grouped[g]
            if pos:
                if g in counts:
                    self.encode_partial(g, [rows[i] for i in pos], c0, parts[g], counts[g])
                else:
                    self.encode_partial(g, [rows[i] for i in pos], c0, parts[g])
            else:
                parts[g].zero_()
            if group is not None:
                handles.append(torch.distributed.all_reduce(parts[g], group=group, async_op=True))

        for g in range(self.G):
            if g not in early:
                run(g)
        if early:
            torch.cuda.current_stream(self.device).wait_event(self._counts_ready)
            for g in early:
                run(g)
        return parts, handles

    def __call__(self, rows, client0=0, total_weight=None, out=None, group=None):
        """out = (sum over groups, in order, of the group partials) / total_weight (default: the
        client count, over all ranks of `group`)."""
        n = rows.shape[0] if torch.is_tensor(rows) else len(rows)
        parts, handles = self.partials(rows, client0, group)
        for h in handles:
            h.wait()
        if total_weight is None:
            world = torch.distributed.get_world_size(group) if group is not None else 1
            total_weight = float(n * world)
        if out is None:
            out = torch.empty(self.D, dtype=torch.float32, device=self.device)
        out.copy_(parts[0])
        for g in range(1, self.G):
            out.add_(parts[g])
        # a device-tensor divisor: torch turns a Python-scalar division on the GPU into a multiply
        # by the reciprocal; the fold's contract (and the reference CPU path) is a true fp32 division
        out.div_(torch.tensor(float(total_weight), dtype=torch.float32, device=out.device))
        return out
