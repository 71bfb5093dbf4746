#!/usr/bin/env python3
"""Benchmark: device-resident gradient-codec encode + N-way reduce on MI355X.

BASELINE.json metric: "gradient-codec encode+reduce GB/s (device-resident), [N,D] fp32; % HBM peak".

A step = one simulated uplink: every client row of the resident synthetic [N, D] fp32 matrix is
encoded with its codec and the rows are reduced to one [D] direction (flc_encode_reduce, one
call); with --gpus G > 1 every rank holds its own N-row shard (weak scaling, one process per GPU)
and the [D] partial sums are combined with one RCCL all-reduce over xGMI, then divided by the
global client count.

Workloads (BASELINE.json configs; the default is the largest single-GPU config, C3):
  c3  topk:1%   N=1024 / GPU, D=10 M   (ResNet-18-sized)                     [default]
  c2  randk:1%  N=256  / GPU, D=1 M    (device-RNG indices)
  c4  qsgd:127  N=512  / GPU, D=25 M   (C4's per-GPU shard: at --gpus 8 this IS C4, N=4096)
  c5  randk:1% / topk:1% / qsgd:127 by client id mod 3, N=2048 / GPU, D=100 M (at --gpus 8: N=16384);
      384 resident distinct rows (154 GB) replayed through the clients' row pointers (128 per codec
      group: no kernel reads one row twice before ~GBs of other rows evict it); the per-group [D]
      partials are all-reduced asynchronously, overlapping the next group's encode
  reduce  ident N=512 / GPU, D=25 M   (the serverGradient fold alone)

Algorithmic bytes: topk / qsgd / ident 4*N*D + 4*D; randk 4*N*K + 4*D (device-RNG
indices cost no bytes).  value = algorithmic bytes of all ranks / max-over-ranks step time.

roofline: the dominant kernel's algorithmic bytes per step / its summed launch time per step, timed
with HIP events on its launch stream (flc_profile_*) in a second pass of the same K steps right after
the timed region (the event packets between launches would lengthen the timed steps); peak 8.0 TB/s
(MI355X_MICROARCH.md).  traffic: HBM bytes per launch from rocprofv3 PMC passes
(profiles/pmc_<workload>.json, written by profiles/collect_pmc.py), or null.
cpu_baseline: the reference's CPU uplink (oracle/torch_cpu.py: its torch / numpy calls) timed on
this host's cores, rank 0, pattern / compress / fold separately.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_GBS = 8000.0   # MI355X HBM3E spec, MI355X_MICROARCH.md "Chip-level parameters"

WORKLOADS = {
    "c3": dict(spec="topk:1%", n=1024, d=10_000_000, kernel="k_topk_filter", config=2, n_total=1024,
               others=["k_topk_sample", "k_cand_select", "k_chunk_accum"]),
    "c2": dict(spec="randk:1%", n=256, d=1_000_000, kernel="k_randk_gen", config=1, n_total=256,
               others=["k_randk_counts", "k_chunk_accum"]),
    # sparse QSGD path (dither_sparse.hip): one read of every row in k_ds_filter
    "c4": dict(spec="qsgd:127", n=512, d=25_000_000, kernel="k_ds_filter", config=3, n_total=4096,
               others=["k_ds_sample", "k_ds_resolve", "k_ds_accum"]),
    # C5: mixed per-client codec (client i -> specs[i % 3]); a pool of resident distinct rows is
    # replayed through the clients' row pointers (819 GB of distinct rows per GPU would not fit)
    "c5": dict(spec="mixed", specs=["randk:1%", "topk:1%", "qsgd:127"], n=2048, d=100_000_000, pool=384,
               kernel="k_ds_filter", config=4,
               others=["k_topk_filter", "k_randk_counts", "k_randk_fold", "k_ds_accum", "k_chunk_accum"]),
    # the serverGradient fold alone (identity codec), C4's shard shape
    "reduce": dict(spec="ident", n=512, d=25_000_000, kernel="k_reduce_vec", config=3, n_total=4096, others=[]),
}


def algorithmic_bytes(spec, n, d, k, specs=None):
    if specs:                                  # mixed: client i uses specs[i % G]; one [D] result
        G = len(specs)
        total = 4 * d
        for g, sp in enumerate(specs):
            ng = len(range(g, n, G))
            kg = math.ceil(0.01 * d)
            total += algorithmic_bytes(sp, ng, d, kg) - 4 * d
        return total
    if spec.startswith("randk"):
        return 4 * n * k + 4 * d
    return 4 * n * d + 4 * d


def kernel_bytes(kernel, n, d, k):
    """Algorithmic bytes one launch of the dominant kernel must move."""
    if kernel == "k_randk_fold":
        return 4 * n * k + 4 * d    # device RandK, long rows: gather K values per row, write the [D] result
    if kernel == "k_randk_gen":
        return 4 * n * k            # device RandK, short rows: gather K values per row (into the fold's lists)
    if kernel == "k_randk_coarse":
        return 8 * n * k            # compat RandK (one chunk per superchunk): gather K values per row + write them
    if kernel in ("k_ew_accum_vec", "k_reduce_vec"):
        return 4 * n * d + 4 * d    # read every row once, write the [D] result
    return 4 * n * d                # k_topk_filter / k_ds_filter: read every row once


def cpu_baseline(spec, d, n_job, budget_s=10.0, specs=None):
    """The reference's CPU uplink on this host: oracle/torch_cpu.py issues the
    reference's own torch / numpy calls (generateCompressPattern, compressVector, serverGradient's
    fold) on CPU tensors, with torch's intra-op threads = the host cores this job may use.  Phases
    timed separately per client over a bounded sample (about budget_s of work); `value` is the
    metric's algorithmic bytes of the sample / the sample's pattern + compress + fold time, and the
    time for the bench's N clients is extrapolated linearly (labelled)."""
    from oracle.torch_cpu import time_uplink
    affinity = len(os.sched_getaffinity(0))
    # the job's CPU share: OMP_NUM_THREADS when the launcher sets it (16 per GPU on the MI355X
    # boxes, whose affinity mask shows the whole machine), else every CPU in the affinity mask
    threads = min(affinity, int(os.environ.get("OMP_NUM_THREADS") or affinity))
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        r = time_uplink(specs or [spec], d, budget_s)
    finally:
        torch.set_num_threads(prev)
    n = r["clients"]
    t = r["pattern_s"] + r["compress_s"] + r["fold_s"]
    k = math.ceil(0.01 * d)
    cpu_model = None
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), None)
    except OSError:
        pass
    per = {ph: round(r[ph + "_s"] / n * 1e3, 3) for ph in ("pattern", "compress", "fold")}
    return {"value": round(algorithmic_bytes(spec, n, d, k, specs) / t / 1e9, 4), "unit": "GB/s", "cores": threads,
            "kind": "port",
            "ms_per_client": per,
            "value_encode_fold_only": round(algorithmic_bytes(spec, n, d, k, specs) /
                                            (r["compress_s"] + r["fold_s"]) / 1e9, 4),
            "extrapolated_s_for_bench_N": {"clients": n_job, "seconds": round(t / n * n_job, 1),
                                           "note": "linear in clients (labelled extrapolation)"},
            # the host the baseline ran on
            "host": {"cpu_model": cpu_model, "affinity_cpus": affinity, "torch_threads": threads},
            "sample": f"oracle/torch_cpu.py (the reference's torch calls) "
                      f"{'/'.join(specs) if specs else spec}: numpy-stream patterns, compressVector, "
                      f"serverGradient fold of {n} clients x D={d} ({t:.1f} s, {threads} torch threads)"}


def read_ceiling(rows, out, reps=3):
    """Same-process, same-allocation plain read of the bench rows: the serverGradient fold
    (k_reduce_vec: every row read once with nontemporal float4 loads, the [D] sum written) over
    the resident matrix, timed with HIP events after the timed region.  Separates "slow box or
    unlucky physical placement" from "slower kernel": the dominant kernel's rate is also reported
    as a fraction of this."""
    from flpytorch_amd import aggregation as ag
    n, d = rows.shape
    ag.reduce_rows(out, rows, relative=False, out=out)          # warm (out is overwritten by each call)
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ag.reduce_rows(out, rows, relative=False, out=out)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    return {"kernel": "k_reduce_vec", "rows": n, "bytes": 4 * n * d + 4 * d, "ms": round(best, 4),
            "GBps": round((4 * n * d + 4 * d) / (best * 1e-3) / 1e9, 1)}


def e2e(args):
    """Host-resident uplink: rows in pinned host memory -> H2D -> flc_encode_reduce -> D2H, one GPU.
    The rows are streamed in blocks of `blk` clients on two streams so the H2D copy of block k+1
    overlaps the encode of block k; partial sums (divisor 1.0) are folded on device."""
    from flpytorch_amd import aggregation as ag
    wl = dict(WORKLOADS[args.workload])
    n = args.n or 64
    d = args.d or wl["d"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comp = ag.initCompressor(wl["spec"], d)
    k = getattr(comp, "K", 0) or 0
    g = torch.Generator(device=dev).manual_seed(5)
    blk = 8
    host = torch.empty((n, d), dtype=torch.float32, pin_memory=True)
    for i in range(0, n, blk):
        host[i:i + blk].copy_(torch.randn((min(blk, n - i), d), generator=g, device=dev))
    bufs = [torch.empty((blk, d), dtype=torch.float32, device=dev) for _ in range(2)]
    part = torch.empty(d, dtype=torch.float32, device=dev)
    acc = torch.empty(d, dtype=torch.float32, device=dev)
    out_host = torch.empty(d, dtype=torch.float32, pin_memory=True)
    red = ag.UplinkReducer(comp, device=dev, seed=7)
    copy_s, comp_s = torch.cuda.Stream(), torch.cuda.current_stream()

    def step():
        evs = []
        for b, i in enumerate(range(0, n, blk)):
            buf = bufs[b % 2]
            m = min(blk, n - i)
            with torch.cuda.stream(copy_s):
                if b >= 2:
                    copy_s.wait_event(evs[b - 2])        # buffer free again
                buf[:m].copy_(host[i:i + m], non_blocking=True)
                ready = torch.cuda.Event()
                ready.record(copy_s)
            comp_s.wait_event(ready)
            red(buf[:m], out=part if i else acc, client0=i, divisor=1.0)
            if i:
                acc.add_(part)
            done = torch.cuda.Event()
            done.record(comp_s)
            evs.append(done)
        acc.div_(float(n))
        out_host.copy_(acc, non_blocking=True)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    moved = 4 * n * d + 4 * d
    print(json.dumps({"mode": "end-to-end host->device->host", "codec": wl["spec"], "clients": n, "D": d, "K": k,
                      "ms_per_step": round(dt * 1e3, 3), "pcie_inclusive_GBps": round(moved / dt / 1e9, 2),
                      "note": "rows start in pinned host memory; 2-stream H2D/encode overlap, blocks of 8 clients"}))


def wire(args):
    """Server side from the wire format: N client payloads already in HBM
    (qsgd:127 -> 1 byte per element + 16-B header, C4's shard shape by default) decoded and folded
    into the [D] mean (flc_unpack_reduce).  Reported on its own line, never as `value`."""
    from flpytorch_amd import _lib
    from flpytorch_amd import aggregation as ag
    wl = dict(WORKLOADS[args.workload])
    n, d = args.n or wl["n"], args.d or wl["d"]
    spec = wl["spec"] if wl["spec"] != "mixed" else "qsgd:127"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    pool = min(n, 16)
    gen = torch.Generator(device=dev).manual_seed(77)
    comps = []
    c0 = ag.initCompressor(spec, d)
    ld = c0.payloadBytes()
    pay = torch.empty((n, ld), dtype=torch.uint8, device=dev)
    x = torch.empty(d, dtype=torch.float32, device=dev)
    rs = np.random.RandomState(5)
    for i in range(pool):
        x.normal_(generator=gen)
        c = ag.initCompressor(spec, d)
        c.device_rng = (20241015, i)
        c.compressPayload(x, out=pay[i])
        comps.append(c)
    for i in range(pool, n):
        pay[i].copy_(pay[i % pool])
    red = ag.PayloadReducer(c0, device=dev)
    out = torch.empty(d, dtype=torch.float32, device=dev)
    for _ in range(args.warmup):
        red(pay, d=d, out=out)
    torch.cuda.synchronize()
    _lib.profile_enable(True)
    _lib.profile_collect("k_unpack_accum")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        red(pay, d=d, out=out)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    _lib.profile_enable(False)
    kms, kn = _lib.profile_collect("k_unpack_accum")
    moved = n * ld + 4 * d
    kern = moved / (kms / max(kn, 1) * 1e-3) / 1e9 if kn else None
    print(json.dumps({"mode": "server decode+reduce from wire payloads (flc_unpack_reduce)", "codec": spec,
                      "clients": n, "D": d, "payload_bytes_per_client": ld,
                      "dense_bytes_per_client": 4 * d, "ms_per_step": round(dt * 1e3, 3),
                      "payload_GBps": round(moved / dt / 1e9, 1),
                      "dense_equivalent_GBps": round((4 * n * d + 4 * d) / dt / 1e9, 1),
                      "kernel": "k_unpack_accum", "kernel_GBps": round(kern, 1) if kern else None,
                      "note": f"{pool} distinct payloads replicated to {n} rows; device-RNG draws"}))


def e2e_wire(args):
    """Host-resident messages: N client payloads (the wire format, e.g. 1 byte per element for
    qsgd:127) in pinned host memory -> H2D -> flc_unpack_reduce -> D2H of the [D] mean.  The
    server side of a simulator whose clients ship their encoded messages instead of fp32 rows;
    blocks of `blk` payloads on two streams, the copy of block k+1 under the fold of block k."""
    from flpytorch_amd import aggregation as ag
    wl = dict(WORKLOADS[args.workload])
    n = args.n or 64
    d = args.d or wl["d"]
    spec = wl["spec"] if wl["spec"] != "mixed" else "qsgd:127"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    c0 = ag.initCompressor(spec, d)
    ld = c0.payloadBytes()
    gen = torch.Generator(device=dev).manual_seed(5)
    host = torch.empty((n, ld), dtype=torch.uint8, pin_memory=True)
    x = torch.empty(d, dtype=torch.float32, device=dev)
    for i in range(n):
        x.normal_(generator=gen)
        c = ag.initCompressor(spec, d)
        c.device_rng = (20241015, i)
        host[i].copy_(c.compressPayload(x))
    blk = 8
    bufs = [torch.empty((blk, ld), dtype=torch.uint8, device=dev) for _ in range(2)]
    part = torch.empty(d, dtype=torch.float32, device=dev)
    acc = torch.empty(d, dtype=torch.float32, device=dev)
    out_host = torch.empty(d, dtype=torch.float32, pin_memory=True)
    red = ag.PayloadReducer(c0, device=dev)
    copy_s, comp_s = torch.cuda.Stream(), torch.cuda.current_stream()
    div = torch.tensor(float(n), dtype=torch.float32, device=dev)

    def step():
        evs = []
        for b, i in enumerate(range(0, n, blk)):
            buf = bufs[b % 2]
            m = min(blk, n - i)
            with torch.cuda.stream(copy_s):
                if b >= 2:
                    copy_s.wait_event(evs[b - 2])
                buf[:m].copy_(host[i:i + m], non_blocking=True)
                ready = torch.cuda.Event()
                ready.record(copy_s)
            comp_s.wait_event(ready)
            red(buf[:m], d=d, out=part if i else acc, divisor=1.0)
            if i:
                acc.add_(part)
            done = torch.cuda.Event()
            done.record(comp_s)
            evs.append(done)
        acc.div_(div)
        out_host.copy_(acc, non_blocking=True)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    moved = n * ld + 4 * d
    print(json.dumps({"mode": "end-to-end host->device->host from wire payloads", "codec": spec, "clients": n,
                      "D": d, "payload_bytes_per_client": ld, "ms_per_step": round(dt * 1e3, 3),
                      "pcie_inclusive_payload_GBps": round(moved / dt / 1e9, 2),
                      "dense_equivalent_GBps": round((4 * n * d + 4 * d) / dt / 1e9, 2),
                      "note": "payloads in pinned host memory; 2-stream H2D/fold overlap, blocks of 8 clients"}))


def shift(args):
    """The compressed algorithms' client step on one client row, fused in one
    call (Compressor.compressShift -> flc_encode_shift) against the same step as the reference
    writes it in torch on the GPU (compressVector(a - b), then the scalar ops):
      diana   m = C(g - h); h' = h + alpha m                    algorithms.py:1383-1391
      ef21    g' = g_prev + C(g - g_prev) * mult                algorithms.py:1506-1517
      marina  g' = g_prev + C(g_cur - g_prev_x)                 algorithms.py:537
    Device-RNG draws.  Bytes of the fused step: a, b read, msg written (+ h read and written for
    diana, + base read for ef21 / marina).  Own line, not `value`."""
    from flpytorch_amd import aggregation as ag
    wl = dict(WORKLOADS[args.workload])
    d = args.d or wl["d"]
    spec = wl["spec"] if wl["spec"] != "mixed" else "qsgd:127"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = torch.Generator(device=dev).manual_seed(11)
    a = torch.randn(d, generator=g, device=dev)
    b = torch.randn(d, generator=g, device=dev) * 0.5
    base = torch.randn(d, generator=g, device=dev)
    c = ag.initCompressor(spec, d)
    c.device_rng = (20241015, 3)
    alpha = 1.0 / (1.0 + c.getW()) if c.isUnbiasedCompressor() else 1.0
    msg_out = torch.empty(d, device=dev)
    h_out = torch.empty(d, device=dev)
    algo = args.shift
    if algo == "diana":
        fused = lambda: c.compressShift(a, b, alpha=alpha, shift=b, shift_out=h_out, out=msg_out)
        torch_step = lambda: (lambda m: (m, b + alpha * m))(c.compressVector(a - b))
        moved = 4 * d * 5                     # a, b (= h) read; msg, h' written; h read for the update
    elif algo == "ef21":
        fused = lambda: c.compressShift(a, b, scale=alpha, base=b, out=msg_out)
        torch_step = lambda: b + c.compressVector(a - b) * alpha
        moved = 4 * d * 3
    else:
        fused = lambda: c.compressShift(a, b, base=base, out=msg_out)
        torch_step = lambda: base + c.compressVector(a - b)
        moved = 4 * d * 4
    res = {}
    for name, fn in (("fused_flc_encode_shift", fused), ("torch_ops_around_compressVector", torch_step)):
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        res[name] = round((time.perf_counter() - t0) / args.steps * 1e3, 4)
    print(json.dumps({"mode": f"{algo} client step (compressShift) vs the reference's torch expression on the GPU",
                      "codec": spec, "D": d, "ms_per_step": res,
                      "fused_GBps": round(moved / (res["fused_flc_encode_shift"] * 1e-3) / 1e9, 1),
                      "bytes_per_step": moved,
                      "note": "device-RNG draws; bytes: the step's vectors read / written once (dithering adds a norm pass)"}))


def dropin(args):
    """The drop-in path as the reference's algorithms drive it after install(): every client's
    Compressor.compressVector (generateCompressPattern on the caller's numpy stream first: compat
    mode, the reference's own draws) and then the serverGradient fold of the N dense outputs
    (reduce_rows) — against the fused uplink (UplinkReducer) on the same rows.  Own line, not value.

    roofline: the bytes the protocol mandates (algorithms.py:1735-1745 -> compressors.py:218-371,
    then 1753-1768): a compressVector reads x and writes the dense [D] output (8 D; dithering in
    compat mode also reads the float64 uniforms, 8 D), the fold reads the N dense outputs and
    writes gs (4 N D + 4 D).  Device time of one compressVector from HIP events around the call
    on its stream (many calls, mean), of the fold likewise."""
    from flpytorch_amd import _lib
    from flpytorch_amd import aggregation as ag
    _lib.check_provenance()
    wl = dict(WORKLOADS[args.workload])
    n = args.n or 32
    d = args.d or wl["d"]
    spec = wl["spec"] if wl["spec"] != "mixed" else "qsgd:127"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    gen = torch.Generator(device=dev).manual_seed(9)
    rows = torch.randn(n, d, generator=gen, device=dev)
    x = torch.zeros(d, device=dev)
    comps = [ag.initCompressor(spec, d) for _ in range(n)]
    for c in comps:
        # "torch_cpu": the reference's own norm bits (torch's CPU order, k_norm_torch) — the price
        # of bit-exact dithering through install()
        c.norm_mode = args.norm_mode
    rs = np.random.RandomState(123)
    dither = spec.startswith(("qsgd", "std.dithering", "nat.dithering", "natural", "terngrad"))
    for i in range(n):                              # compat patterns drawn once (host numpy stream)
        comps[i].generateCompressPattern(rs, "cuda", i, {})

    def per_client(patterns=True):
        outs = []
        for i in range(n):
            if patterns:
                comps[i].generateCompressPattern(rs, "cuda", i, {})
            outs.append(comps[i].compressVector(rows[i]))
        return ag.reduce_rows(x, outs, relative=False)

    def dev_time(fn, reps):
        """mean device ms of fn() (HIP events on the current stream, which the library launches on)"""
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / reps

    # one compressVector at a time (the reference's serial round order), patterns resident
    if dither:
        for c in comps:                             # the uniforms on the device once (the protocol's lazy .to)
            c.testp = c.testp.to(dev)
    # every client's row in turn (rows differ in their selection work, e.g. ties at the K-th key):
    # the mean device time of one call
    def all_rows():
        for i in range(n):
            comps[i].compressVector(rows[i])
    reps = max(args.steps, 20)
    cv_ms = dev_time(all_rows, max(reps // n, 3)) / n
    outs = [comps[i].compressVector(rows[i]) for i in range(n)]
    fold_ms = dev_time(lambda: ag.reduce_rows(x, outs, relative=False), max(args.steps, 5))
    cv_bytes = 8 * d + (8 * d if dither else 0)
    fold_bytes = 4 * n * d + 4 * d

    def rate(b, ms):
        gbs = b / (ms * 1e-3) / 1e9
        return {"ms": round(ms, 4), "bytes": b, "GBps": round(gbs, 1), "frac": round(gbs / PEAK_GBS, 4)}

    red = ag.UplinkReducer(ag.initCompressor(spec, d), device=dev, seed=5)
    res = {}
    for name, fn in [("per_client_compat_incl_patterns", lambda: per_client(True)),
                     ("per_client_encode_and_fold_only", lambda: per_client(False)),
                     ("fused_uplink_device_rng", lambda: red(rows))]:
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        res[name] = round((time.perf_counter() - t0) / args.steps * 1e3, 3)
    # per-kernel device time of one compressVector, over every client's row (flc_profile scopes)
    kernels = ["k_topk_sample", "k_topk_filter", "k_cand_select", "k_topk_exact_rows", "k_chunk_accum",
               "k_norm_partials", "k_ew_accum_vec", "k_ew_encode", "k_randk_scatter_dev", "k_assign_scatter",
               "k_assign_finish", "k_lone_dither", "k_lone_resident", "k_norm_torch", "k_tn_sums", "k_tn_maps", "k_tn_walk"]
    _lib.profile_enable(True)
    for k in kernels:
        _lib.profile_collect(k)
    for _ in range(max(10 // n, 2)):
        all_rows()
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    per_kernel = {}
    for k in kernels:
        ms, cnt = _lib.profile_collect(k)
        if cnt:
            per_kernel[k] = round(ms / cnt * 1e3, 2)
    cv = rate(cv_bytes, cv_ms)
    # PMC traffic of the compressVector kernel (tools/collect_pmc.py --dropin), when its pass is on file
    cv_traffic, cv_kernel = None, None
    pmc = os.path.join(ROOT, "profiles", f"pmc_dropin_{args.workload}.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            pj = json.load(f)
        cv_kernel = pj.get("kernel")
        # the same compressVector kernel at the same D
        if cv_kernel and any(cv_kernel in k for k in per_kernel) and pj.get("d") == d and args.norm_mode == "exact":
            cv_traffic = pj.get("hbm_bytes_per_launch")
    print(json.dumps({"metric": "drop-in compressVector + serverGradient fold, device time; % HBM peak",
                      "mode": "drop-in path (compressVector per client + serverGradient fold) vs fused uplink",
                      "codec": spec, "clients": n, "D": d, "norm_mode": args.norm_mode,
                      "roofline": {"bound": "hbm", "kernel": "compressVector (one row)", "achieved": cv["GBps"],
                                   "peak": PEAK_GBS, "unit": "GB/s", "frac": cv["frac"], "traffic": cv_traffic,
                                   "traffic_unit": "HBM bytes per launch of " + str(cv_kernel) + " (rocprofv3 PMC, profiles/)",
                                   "traffic_over_algorithmic": round(cv_traffic / cv_bytes, 4) if cv_traffic else None,
                                   "bytes_per_call": cv_bytes, "us_per_call": round(cv_ms * 1e3, 2),
                                   "per_kernel_us": per_kernel,
                                   "bytes_note": "read x + write the dense output (8 D)"
                                                 + (" + the float64 uniforms (8 D)" if dither else "")},
                      "fold": rate(fold_bytes, fold_ms),
                      "round_device_ms": round(n * cv_ms + fold_ms, 4),
                      "ms_per_round": res,
                      "note": "compat mode draws the reference's numpy stream on the host (MT19937 in C++) "
                              "and uploads it; the second line reuses the drawn patterns"}))


def dist_info(dist, dev, d, reps=5):
    """What the process group really was, so that "RCCL saw N ranks" can be
    checked from the bench line itself: the group's own world size and backend, every rank's host,
    device index and PCI bus id (all_gather_object), the RCCL version torch links, and the time of
    the step's exchange alone — an all-reduce of the [D] fp32 partial, timed after the bench's
    timed region (max over ranks), with its ring bus bandwidth 2 (G-1)/G x bytes / t.  Collective:
    every rank calls it.  Works on the gloo backend with CPU tensors (tests/test_bench_launcher.py)."""
    import socket
    import torch
    g = dist.get_world_size()
    backend = dist.get_backend()
    me = {"rank": dist.get_rank(), "host": socket.gethostname(), "device": None, "pci_bus_id": None}
    if dev.type == "cuda":
        me["device"] = torch.cuda.current_device()
        props = torch.cuda.get_device_properties(dev)
        bus = getattr(props, "pci_bus_id", None)
        me["pci_bus_id"] = (f"{getattr(props, 'pci_domain_id', 0):04x}:{bus:02x}:{getattr(props, 'pci_device_id', 0):02x}"
                            if isinstance(bus, int) else bus)
        me["device_name"] = props.name
    ranks = [None] * g
    dist.all_gather_object(ranks, me)
    ver = None
    if backend == "nccl":
        try:
            v = torch.cuda.nccl.version()
            ver = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
        except Exception as e:  # noqa: BLE001 — reported, not fatal
            ver = f"unavailable ({type(e).__name__})"
    t = torch.zeros(d, dtype=torch.float32, device=dev)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    dist.all_reduce(t)                                   # warm (communicator set up)
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        dist.all_reduce(t)
    sync()
    ms = (time.perf_counter() - t0) / reps * 1e3
    m = torch.tensor([ms], dtype=torch.float64, device=dev)
    dist.all_reduce(m, op=dist.ReduceOp.MAX)
    ms = float(m.item())
    nbytes = 4 * d
    return {"pg_world_size": g, "backend": backend, "rccl_version": ver, "ranks": ranks,
            "distinct_devices": len({(r["host"], r["pci_bus_id"], r["device"]) for r in ranks}),
            "allreduce_bytes": nbytes, "allreduce_ms": round(ms, 4),
            "allreduce_busbw_GBps": round(2.0 * (g - 1) / g * nbytes / (ms * 1e-3) / 1e9, 3) if ms > 0 else None}


def strong_block(encode_partial, fold, block_rows, n_total, d, dev, steps, warmup, group=None):
    """The north_star's scaling measurement on every line: C4 at FIXED N
    (n_total clients, qsgd:127 on the GPU) in the 8 fixed client blocks of sharding.py, rank r of G
    owning blocks r*8/G .., every block encoded into its own exact partial, the partials combined in
    block order ("ordered": all-to-all + block-order fold + all-gather), so the [D] result has the
    same bits at G = 1, 2, 4, 8.  Every rank holds the same resident block of rows (block_rows:
    n_total / 8 rows, identical on every rank) and replays it for each of its blocks with the
    block's own client ids (its own device-RNG draws): the work of a block does not depend on G.
    Returns ms per step (max over ranks, barrier + sync around exactly `steps` steps), the
    whole-job rate 4 n_total D + 4 D bytes / step, and the sha256 of the result's bytes, from which
    a SCALE run reads both the speed-up and the G-invariance.  Collective: every rank calls it."""
    import hashlib
    import torch.distributed as dist
    from flpytorch_amd.sharding import N_BLOCKS, ShardedUplink, rank_clients
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if world > 1 else 0
    r_lo, r_hi = rank_clients(n_total, world, rank)
    uplink = ShardedUplink(encode_partial, group=group, mode="ordered", fold=fold)
    out = torch.empty(d, dtype=torch.float32, device=dev)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier(group)

    def step():
        uplink(lambda lo, hi: block_rows[:hi - lo], client0=r_lo, total_weight=float(n_total), n_clients=n_total,
               out=out, d=d, device=dev)
    for _ in range(warmup):
        step()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        elapsed = float(t.item())
    ms = elapsed / steps * 1e3
    nbytes = 4 * n_total * d + 4 * d
    digest = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()
    return {"workload": f"C4 qsgd:127 N={n_total} (fixed) D={d}, {N_BLOCKS} client blocks, ordered combine",
            "n_gpus": world, "clients_total": n_total, "clients_per_gpu": r_hi - r_lo, "steps": steps, "warmup": warmup,
            "ms_per_step": round(ms, 4), "value_GBps": round(nbytes / (ms * 1e-3) / 1e9, 2),
            "pct_hbm_peak_per_gpu": round(100.0 * nbytes / (ms * 1e-3) / 1e9 / world / PEAK_GBS, 2),
            "result_sha256": digest,
            "scaling": "strong (fixed N; speed-up = this line's ms_per_step at G=1 / at G)",
            "rows": f"{block_rows.shape[0]} resident rows per GPU (one fixed-seed block, the same on every rank) "
                    "replayed for each of the rank's blocks with the block's client ids"}


def launch_ranks(gpus, cmd, poll_s=0.2, grace_s=10.0):
    """One process per GPU without an outside launcher (`python3 bench.py --gpus G`): G fresh
    children of ``cmd``, each with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in its
    environment (torch.distributed.run's contract, rendezvous on 127.0.0.1), started before this
    process has made any GPU call — the parent never re-execs itself and never touches the GPU.
    Waits for every rank; when one fails the others are terminated (then killed after grace_s) so
    a rank stuck in a collective cannot hang the job.  Returns 0, or the first failing rank's exit
    status (a signal as 128 + signo).  Replaces the reference's thread-per-device dispatch
    (thread_pool.py:56-67) with one process per GPU."""
    import signal
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(gpus), LOCAL_WORLD_SIZE=str(gpus),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env))
    status, failed_at = 0, None
    while True:
        codes = [p.poll() for p in procs]
        for c in codes:
            if c is not None and c != 0 and status == 0:
                status = c if c > 0 else 128 - c
                failed_at = time.monotonic()
                for p in procs:
                    if p.poll() is None:
                        p.send_signal(signal.SIGTERM)
        if all(c is not None for c in codes):
            return status
        if failed_at is not None and time.monotonic() - failed_at > grace_s:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        time.sleep(poll_s)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    # --clients / --dim: the spellings to use under torch.distributed.run (its parser takes "--n" as an
    # ambiguous abbreviation of its own options)
    ap.add_argument("--n", "--clients", dest="n", type=int, default=None, help="override clients per GPU")
    ap.add_argument("--d", "--dim", dest="d", type=int, default=None, help="override D")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-counts-overlap", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--dist", choices=["normal", "heavy"], default="normal",
                    help="synthetic rows: N(0,1) (default) or N(0,1) * 10^U(-3,3) (SURVEY 8d)")
    ap.add_argument("--shift", choices=["diana", "ef21", "marina"], default=None,
                    help="the compressed algorithms' client step on one row (flc_encode_shift) vs torch ops")
    ap.add_argument("--step-times", action="store_true", help="per-step times (HIP events) on stderr")
    ap.add_argument("--row-groups", type=int, default=None,
                    help="sparse QSGD / TopK execution hint: fold row group g while group g+1 is filtered")
    ap.add_argument("--compat", action="store_true",
                    help="compat-mode patterns: the reference's numpy-stream RandK indices / dithering uniforms, "
                         "resident in HBM and read by the kernels (their bytes counted)")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: N clients per GPU; strong: the workload's fixed round size (C4: N=4096) in 8 "
                         "fixed client blocks over the GPUs, combined in block order (G-invariant)")
    ap.add_argument("--dropin", action="store_true",
                    help="per-client compressVector + serverGradient fold (the install() path) vs the fused uplink")
    ap.add_argument("--wire", action="store_true",
                    help="server side from the wire format: decode+reduce of N resident payloads (own line, not value)")
    ap.add_argument("--norm-mode", default="exact", choices=["exact", "torch_cpu"],
                    help="--dropin: Compressor.norm_mode of the dithering codecs (torch_cpu: the reference's norm bits)")
    ap.add_argument("--alloc", choices=["contiguous", "default"], default="contiguous",
                    help="the resident rows' HBM: one physically contiguous range (flc_rows_alloc) or torch's allocator")
    ap.add_argument("--no-strong-c4", action="store_true",
                    help="skip the strong_c4 block (C4 at fixed N=4096, ordered combine) of the default line")
    ap.add_argument("--strong-steps", type=int, default=5, help="timed steps of the strong_c4 block")
    ap.add_argument("--e2e", action="store_true",
                    help="end-to-end: client rows start in pinned host memory, the [D] result lands in host memory "
                         "(H2D + encode+reduce + D2H per step; PCIe-bound; reported in DESIGN.md, never as value)")
    args = ap.parse_args()
    if args.shift:
        return shift(args)
    if args.dropin:
        return dropin(args)
    if args.e2e and args.wire:
        return e2e_wire(args)
    if args.e2e:
        return e2e(args)
    if args.wire:
        return wire(args)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no outside launcher: this process starts the G ranks itself (nothing has touched the GPU yet)
        sys.exit(launch_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))

    wl = dict(WORKLOADS[args.workload])
    if args.n:
        wl["n"] = args.n
    if args.d:
        wl["d"] = args.d
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # rehearsal of the multi-rank path on a one-GPU box (never the measured configuration):
    # FLC_BENCH_SHARE_GPU=1 puts every rank on cuda:0, FLC_BENCH_BACKEND=gloo swaps RCCL for gloo
    if os.environ.get("FLC_BENCH_SHARE_GPU") == "1":
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        # one node (the bench contract): RCCL's bootstrap on loopback unless the caller chose
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        backend = os.environ.get("FLC_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from flpytorch_amd import _lib
    from flpytorch_amd import aggregation as ag
    build_id = _lib.check_provenance()            # the .so must be the one this tree builds

    n, d, spec = wl["n"], wl["d"], wl["spec"]
    specs = wl.get("specs")
    mixed = specs is not None
    k = math.ceil(0.01 * d) if mixed else (getattr(ag.initCompressor(spec, d), "K", 0) or 0)
    strong = args.scaling == "strong"
    if strong:
        # fixed N for every G: the round's n_total clients in 8 fixed blocks,
        # rank r of G owns blocks r*8/G ..; each block folded into its own exact partial, the 8
        # partials combined in block order (G-invariant bits).  A rank holds its clients' rows when
        # they fit (160 GB), else one block's rows, replayed for every block it owns (each block
        # with its own client ids, hence its own device-RNG draws) — C4's 1-GPU point replays the
        # resident 512-row shard 8x
        if mixed:
            raise SystemExit("--scaling strong: not for the mixed workload (c5)")
        from flpytorch_amd.sharding import N_BLOCKS, ShardedUplink, product_fold, product_partial, rank_clients
        n_total = wl["n_total"] if not args.n else args.n
        r_lo, r_hi = rank_clients(n_total, world, rank)
        n = r_hi - r_lo
        block = -(-n_total // N_BLOCKS)
        replay = n * d * 4 > 160e9
        n_dist = block if replay else n
    # synthetic rows ~ N(0, 1) fp32, seeded per rank (device generator; never leaves HBM)
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)
    if not strong:
        n_dist = min(n, wl["pool"]) if mixed else n
    # the resident client-update matrix in physically contiguous HBM (flpytorch_amd.resident: the
    # default allocation's fragments read 6-10 % slower in places, more translation misses)
    from flpytorch_amd.resident import resident_rows
    rows, rows_alloc = resident_rows(n_dist, d, device=dev, contiguous=args.alloc == "contiguous")
    for i in range(0, n_dist, 64):
        rows[i:i + 64].normal_(generator=gen)
        if args.dist == "heavy":
            # SURVEY §8d's second distribution: N(0,1) * 10^U(-3,3), a wide dynamic range that moves
            # the TopK thresholds and the QSGD level mix (heavy-tailed norm samples)
            e = torch.empty_like(rows[i:i + 64]).uniform_(-3.0, 3.0, generator=gen)
            rows[i:i + 64].mul_(torch.pow(10.0, e))
            del e
    out = torch.empty(d, dtype=torch.float32, device=dev)
    client0 = rank * n
    compat_kw, compat_bytes, compat_note = {}, 0, None
    if args.compat and spec.startswith("randk"):
        wl["kernel"], wl["others"] = "k_randk_coarse", ["k_randk_fine", "k_chunk_accum"]
    if args.compat and not spec.startswith("randk") and wl["kernel"] != "k_ds_filter":
        # float64 uniforms of the dense two-pass codecs (norm pass, then the encode pass reading row
        # + uniforms): the encode pass is the dominant kernel.  QSGD (k_ds_filter) reads the
        # uniforms beside the rows in its single pass.
        wl["kernel"], wl["others"] = "k_ew_accum_vec", ["k_norm_partials"]
    if args.compat:
        # compat mode: the reference's numpy-stream patterns, drawn on the host (the
        # C++ MT19937 restatement, bit-exact) before the timed region and resident in HBM; the
        # kernels read them: RandK int64 indices (+8 N K bytes), dithering float64 uniforms (+8 N D)
        if world > 1 or mixed or strong:
            raise SystemExit("--compat: single-GPU, single-codec workloads")
        rs = np.random.RandomState(123)
        t0 = time.perf_counter()
        if spec.startswith("randk"):
            idx = np.empty((n, k), dtype=np.int64)
            for i in range(n):
                idx[i] = ag.stream_choice(rs, d, k)
                ag.stream_randint31(rs)
            compat_kw["randk_idx"] = torch.from_numpy(idx).to(dev)
            compat_bytes = 8 * n * k
            compat_note = f"host numpy-stream choice(D, K) for {n} clients: {(time.perf_counter() - t0) * 1e3:.0f} ms"
        elif spec.startswith(("qsgd", "std_dithering", "natural", "terngrad")):
            # float64 uniforms of `pool` clients drawn from the stream, replicated over the N rows
            # (N x D x 8 B resident; the numbers do not change the kernels' work)
            pool = min(n, 16)
            uni = torch.empty((n, d), dtype=torch.float64, device=dev)
            host = np.empty(d, dtype=np.float64)
            for i in range(pool):
                ag.stream_rand(rs, d, out=host)
                ag.stream_randint31(rs)
                uni[i].copy_(torch.from_numpy(host))
            for i in range(pool, n):
                uni[i].copy_(uni[i % pool])
            compat_kw["uniforms"] = uni
            compat_bytes = 8 * n * d
            compat_note = (f"host numpy-stream rand(D) for {pool} clients ({(time.perf_counter() - t0) / pool * 1e3:.0f} "
                           f"ms per client), replicated over the {n} rows")
        else:
            raise SystemExit(f"--compat: {spec} draws no pattern")
        torch.cuda.synchronize()
    if mixed:
        row_list = [rows[i % n_dist] for i in range(n)]
        up = ag.MixedUplink(specs, d, seed=20241015, device=dev)
        if args.no_counts_overlap:
            up.counts_groups = []            # A/B: the RandK counts inside the call, not beside the filters
        group = None
        if world > 1:
            group = dist.group.WORLD
    else:
        comp = ag.initCompressor(spec, d)
        if args.row_groups:
            comp.row_groups = args.row_groups      # execution hint: the fold of row group g under group g+1's pass
        red = ag.UplinkReducer(comp, device=dev, seed=20241015)

    if strong:
        uplink = ShardedUplink(product_partial(red), group=dist.group.WORLD if world > 1 else None, mode="ordered",
                               fold=product_fold())

        def rows_of(b_lo, b_hi):
            return rows[:b_hi - b_lo] if replay else rows[b_lo - r_lo:b_hi - r_lo]
    elif world > 1 and not mixed:
        from flpytorch_amd.sharding import ShardedUplink, product_partial
        # local partial = sum_i C_i(row_i) in client order (fp32 divisor 1.0 keeps it exact),
        # one RCCL all-reduce of D floats over xGMI, then the global mean
        uplink = ShardedUplink(product_partial(red), mode="allreduce")

    def step():
        if strong:
            uplink(rows_of, client0=r_lo, total_weight=float(n_total), n_clients=n_total, out=out, d=d, device=dev)
        elif mixed:
            up(row_list, client0=client0, total_weight=float(n * world), out=out, group=group)
        elif world == 1:
            red(rows, out=out, client0=client0, **compat_kw)
        else:
            uplink(rows, client0=client0, total_weight=float(n * world), out=out)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    # The timed region: exactly K steps, nothing else on the GPU.  The per-kernel HIP events of the
    # roofline (a begin/end pair around every hot launch, flc_profile_*) are NOT recorded here: each
    # record is a queue packet between launches, and at C3 (~12 launches per step) they lengthened
    # the step by 1.4 % (0.11 ms, same allocation, round 4).
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if args.step_times:
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
        evs[0].record()
    for i in range(args.steps):
        step()
        if args.step_times:
            evs[i + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if args.step_times and rank == 0:
        print(json.dumps({"step_ms": [round(evs[i].elapsed_time(evs[i + 1]), 3) for i in range(args.steps)]}),
              file=sys.stderr)
    # The roofline's kernel times: the same K steps again with the HIP event pair around every
    # launch of the dominant kernel (and the tail kernels), recorded on the stream each is launched
    # on; only kernel durations are read from this pass, never the step time.
    _lib.profile_enable(True)
    for kname in [wl["kernel"]] + wl["others"]:
        _lib.profile_collect(kname)             # drop anything recorded before this pass
    for i in range(args.steps):
        step()
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    kms, klaunch = _lib.profile_collect(wl["kernel"])
    others = {}
    for kname in wl["others"]:
        oms, on = _lib.profile_collect(kname)
        if on:
            others[kname] = round(oms / on, 4)
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ceiling = read_ceiling(rows, out)
    mg = dist_info(dist, dev, d) if world > 1 else None
    strong_c4 = None
    if args.workload == "c3" and not (args.no_strong_c4 or args.compat or strong or args.d):
        # the north_star's fixed-N scaling curve (C4, N=4096) on every default line, G = 1 included:
        # the C3 rows are released first (51.2 GB of C4 block rows + its workspace instead)
        del rows
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        from flpytorch_amd.sharding import N_BLOCKS, product_fold, product_partial
        c4 = WORKLOADS["c4"]
        blk = c4["n_total"] // N_BLOCKS
        g4 = torch.Generator(device=dev).manual_seed(4096)          # the same rows on every rank
        rows4, alloc4 = resident_rows(blk, c4["d"], device=dev, contiguous=args.alloc == "contiguous")
        for i in range(0, blk, 64):
            rows4[i:i + 64].normal_(generator=g4)
        red4 = ag.UplinkReducer(ag.initCompressor(c4["spec"], c4["d"]), device=dev, seed=20241015)
        strong_c4 = strong_block(product_partial(red4), product_fold(), rows4, c4["n_total"], c4["d"], dev,
                                 steps=args.strong_steps, warmup=1, group=dist.group.WORLD if world > 1 else None)
        strong_c4["rows_alloc"] = alloc4
        del rows4

    step_ms = elapsed / args.steps * 1e3
    total_bytes = algorithmic_bytes(spec, n_total, d, k) if strong else algorithmic_bytes(spec, n, d, k, specs) * world
    total_bytes += compat_bytes
    value = total_bytes / (elapsed / args.steps) / 1e9
    # the dominant kernel may run as several launches per step (sparse QSGD: one per row group):
    # its achieved rate is the algorithmic bytes of a step over its summed launch time per step
    # mixed: the dominant kernel serves the qsgd group only
    kb = kernel_bytes(wl["kernel"], len(range(specs.index("qsgd:127"), n, len(specs))) if mixed else n, d, k)
    kb += compat_bytes                     # the dominant kernel reads the resident compat patterns
    kavg_ms = kms / max(klaunch, 1)
    kstep_ms = kms / args.steps
    achieved = kb / (kstep_ms * 1e-3) / 1e9 if klaunch else None
    launches_per_step = klaunch / args.steps if klaunch else 0
    kb_launch = kb / launches_per_step if launches_per_step else None
    line_floor = None
    if wl["kernel"] in ("k_randk_fold", "k_randk_gen"):
        # sparse 4-B gathers fetch whole 128-B lines (profiles/archive/r02/probe_gather_fetch.txt): the
        # gather's physical floor is the expected number of distinct lines touched, x 128 B
        nr = len(range(specs.index("randk:1%"), n, len(specs))) if mixed else n
        line_floor = nr * (d / 32.0) * (1.0 - (1.0 - k / d) ** 32) * 128 + (4 * d if wl["kernel"] == "k_randk_fold" else 0)
    randk_group = None
    if mixed and "randk:1%" in specs:
        # C5's RandK group: counts + list-free fold; algorithmic 4 N_r K + 4 D, the 128-B line floor
        # of its gathers, and the PMC traffic of the fold (profiles/pmc_c5_randk.json)
        nr = len(range(specs.index("randk:1%"), n, len(specs)))
        rk_ms = sum(others.get(kk, 0.0) for kk in ("k_randk_counts", "k_randk_fold"))
        rk_floor = nr * (d / 32.0) * (1.0 - (1.0 - k / d) ** 32) * 128 + 4 * d
        rk_traffic = None
        pmc_rk = os.path.join(ROOT, "profiles", "pmc_c5_randk.json")
        if os.path.exists(pmc_rk):
            with open(pmc_rk) as f:
                pr = json.load(f)
            if pr.get("n") == n and pr.get("d") == d:            # (a pass of this line's shape only)
                rk_traffic = pr.get("hbm_bytes_per_launch")
        if rk_ms:
            randk_group = {"rows": nr, "ms_per_step": round(rk_ms, 4),
                           "algorithmic_GBps": round((4 * nr * k + 4 * d) / (rk_ms * 1e-3) / 1e9, 1),
                           "line_floor_bytes": int(rk_floor),
                           "line_floor_GBps": round(rk_floor / (rk_ms * 1e-3) / 1e9, 1),
                           "fold_traffic_bytes": rk_traffic}
    traffic, traffic_src = None, None
    pmc = os.path.join(ROOT, "profiles", f"pmc_{args.workload}{'_compat' if args.compat else ''}.json")
    if os.path.exists(pmc) and not strong:
        with open(pmc) as f:
            pj = json.load(f)
        # only a PMC pass of this line's shape: the same dominant kernel and
        # pattern source (a compat line's filter also reads the uniforms), rows per GPU, D and
        # launches per step — counters of another shape would price other bytes per launch
        if (wl["kernel"] in pj.get("kernel", "") and bool(pj.get("compat")) == bool(args.compat)
                and pj.get("n") == n and pj.get("d") == d and pj.get("launches_per_step") is not None
                and abs(pj["launches_per_step"] - launches_per_step) < 0.01):
            traffic = pj.get("hbm_bytes_per_launch")
            traffic_src = {"file": os.path.relpath(pmc, ROOT), "n": pj["n"], "d": pj["d"],
                           "launches_per_step": pj["launches_per_step"]}

    if rank == 0:
        cpu = None if args.no_cpu_baseline else cpu_baseline(spec, d, n_total if strong else n * world,
                                                             budget_s=15.0 if mixed else 10.0, specs=specs)
        line = {
            "metric": "gradient-codec encode+reduce GB/s (device-resident), [N,D] fp32; % HBM peak",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(step_ms, 4),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic N(0,1) * 10^U(-3,3)" if args.dist == "heavy" else "synthetic N(0,1)")
                    + f" fp32 rows generated on device (seeded per rank) in {rows_alloc} HBM; "
                    + (f"compat patterns (the reference's numpy stream, resident in HBM; {compat_note})"
                       if args.compat else "device-RNG patterns")
                    + (f"; {n_dist} resident distinct rows replayed through the {n} clients' row pointers, "
                       "each client its own codec (client id mod 3) and device-RNG key" if mixed else "")
                    + (f"; strong scaling: {n_total} clients in {N_BLOCKS} fixed blocks, {n} on this GPU"
                       + (f", one block's {n_dist} rows resident and replayed for each of its blocks (own client ids)"
                          if replay else ", all resident") if strong else ""),
            "config": {"workload": (f"C{wl['config'] + 1} {spec} N={n_total} (fixed) D={d}" if strong else
                                    f"C{wl['config'] + 1} {'/'.join(specs) if mixed else spec} N={n}/GPU D={d}"),
                       "codec": "/".join(specs) if mixed else spec,
                       "clients_per_gpu": n, "clients_total": n_total if strong else n * world, "D": d, "K": k,
                       "rows_alloc": rows_alloc,
                       "parallelism": f"client-shard dp{world}" + (
                           f" + {N_BLOCKS} block partials, all-to-all + block-order fold + all-gather (G-invariant)"
                           if strong else (" + RCCL all-reduce" if world > 1 else ""))},
            "pct_hbm_peak": round(100.0 * value / world / PEAK_GBS, 2),
            # RandK also reports the dense-equivalent rate 4 N D / t (never the roofline)
            "dense_equivalent_GBps": round((4 * n * d + 4 * d) * world / (elapsed / args.steps) / 1e9, 1)
            if (spec.startswith("randk") or mixed) else None,
            "roofline": {"bound": "hbm", "kernel": wl["kernel"],
                         "achieved": round(achieved, 1) if achieved else None, "peak": PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / PEAK_GBS, 4) if achieved else None,
                         # traffic: PMC HBM bytes of ONE launch (the contract's unit, like avg_launch_ms);
                         # beside it the algorithmic bytes of one launch and their ratio, then the step's
                         "traffic": traffic, "traffic_unit": "HBM bytes per launch (rocprofv3 PMC, profiles/)",
                         "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": int(kb_launch) if kb_launch else None,
                         "traffic_over_algorithmic": round(traffic / kb_launch, 4) if (traffic and kb_launch) else None,
                         "traffic_per_step": int(traffic * launches_per_step) if (traffic and klaunch) else None,
                         "bytes_per_step": kb, "kernel_ms_per_step": round(kstep_ms, 4),
                         "kernel_timing": "HIP events around every launch on its stream, in a second pass of the "
                                          "same K steps after the timed region (the events would lengthen the step)",
                         "avg_launch_ms": round(kavg_ms, 4), "launches": klaunch,
                         "other_kernels_avg_ms": others,
                         "read_ceiling_GBps": ceiling["GBps"],
                         "frac_of_read_ceiling": round(achieved / ceiling["GBps"], 4) if achieved else None,
                         "read_ceiling": ceiling,
                         **({"line_floor_bytes_per_step": int(line_floor),
                             "line_floor_GBps": round(line_floor / (kstep_ms * 1e-3) / 1e9, 1) if klaunch else None}
                            if line_floor else {})},
            "cpu_baseline": cpu,
            "build_id": build_id,
        }
        if randk_group:
            line["randk_group"] = randk_group
        if strong_c4:
            line["strong_c4"] = strong_c4
        if mg:
            line["multi_gpu"] = mg
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
