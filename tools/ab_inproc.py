#!/usr/bin/env python3
"""In-process A/B of library builds on ONE resident allocation (GPU box).

The rows' physical placement moves a whole step by up to ~10 % from one allocation (one process)
to the next, which swamps most kernel changes when variants run in separate
processes.  Here every variant (abvar/libflcodec_<tag>.so, "prod" = the product library)
is loaded into one process (_lib.open_variant / _lib.use) and timed on the same rows, rounds
interleaved: the per-variant medians compare kernels at matched placement.  Each round also times
a plain read of the rows (the serverGradient fold) as the allocation's ceiling.

usage: python tools/ab_inproc.py --workload c4 --variants head,prod[,prod:rg4] [--rounds 5] [--steps 5]
Prints one JSON line per (round, variant) and a summary line per variant.

Keep it to three builds per process: each build creates its own side streams, a process has four
hardware queues, and the 4th / 5th build loaded ran every kernel 8-120 % slower in two runs
(profiles/r03/inproc_ab3.txt, inproc_ab4.txt).
"""
import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

WL = {"c3": ("topk:1%", 1024, 10_000_000, ["k_topk_filter", "k_topk_sample", "k_cand_select", "k_chunk_accum"]),
      "c4": ("qsgd:127", 512, 25_000_000, ["k_ds_filter", "k_ds_sample", "k_ds_resolve", "k_ds_accum"]),
      "c2": ("randk:1%", 256, 1_000_000, ["k_randk_gen", "k_randk_counts", "k_chunk_accum"])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4", choices=sorted(WL))
    ap.add_argument("--variants", default="head,prod")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--row-groups", type=int, default=None)
    ap.add_argument("--no-bitcheck", action="store_true", help="probe builds (their outputs are not valid)")
    ap.add_argument("--prof-modes", default="on", help="comma list of on/off: kernel timing events during the steps")
    a = ap.parse_args()
    from flpytorch_amd import _lib
    from flpytorch_amd import aggregation as ag
    spec, n, d, kernels = WL[a.workload]
    n = a.n or n
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    gen = torch.Generator(device=dev).manual_seed(1000)
    rows = torch.empty((n, d), dtype=torch.float32, device=dev)
    for i in range(0, n, 64):
        rows[i:i + 64].normal_(generator=gen)
    out = torch.empty(d, dtype=torch.float32, device=dev)
    # a variant is "<build>" or "<build>:rg<K>" (the same build with the row-group hint K)
    variants = a.variants.split(",")
    builds = sorted({v.split(":")[0] for v in variants})
    if len(builds) > 3:
        print(f"warning: {len(builds)} builds in one process; more than 3 distorted the timing before", file=sys.stderr)
    blibs = {b: _lib.open_variant(b) for b in builds}
    libs = {v: blibs[v.split(":")[0]] for v in variants}
    reds = {}
    modes = a.prof_modes.split(",")
    variants = [f"{v}@{m}" if len(modes) > 1 else v for v in variants for m in modes]
    libs = {v: blibs[v.split("@")[0].split(":")[0]] for v in variants}
    for v in variants:
        comp = ag.initCompressor(spec, d)
        rg = int(v.split("@")[0].split(":rg")[1]) if ":rg" in v else a.row_groups
        if rg:
            comp.row_groups = rg
        reds[v] = ag.UplinkReducer(comp, device=dev, seed=20241015)
    ref = None
    res = {v: [] for v in variants}
    for r in range(a.rounds):
        # the allocation's read ceiling this round (product library)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ag.reduce_rows(out, rows, relative=False, out=out)
        e0.record()
        ag.reduce_rows(out, rows, relative=False, out=out)
        e1.record()
        e1.synchronize()
        read_ms = e0.elapsed_time(e1)
        for v in variants:
            red = reds[v]
            with _lib.use(libs[v]):
                red(rows, out=out)                        # warm (and workspace for this build)
                torch.cuda.synchronize()
                if ref is None:
                    ref = out.clone()
                elif not a.no_bitcheck and not torch.equal(out.view(torch.int32), ref.view(torch.int32)):
                    raise SystemExit(f"variant {v}: output bits differ from {variants[0]}")
                prof = not v.endswith("@off")
                _lib.profile_enable(prof)
                for k in kernels:
                    _lib.profile_collect(k)
                e0.record()
                for _ in range(a.steps):
                    red(rows, out=out)
                e1.record()
                e1.synchronize()
                _lib.profile_enable(False)
                ks = {}
                for k in kernels:
                    ms, cnt = _lib.profile_collect(k)
                    ks[k] = round(ms / a.steps, 4)
            step = e0.elapsed_time(e1) / a.steps
            res[v].append((step, ks))
            print(json.dumps({"round": r, "variant": v, "ms_per_step": round(step, 4), "read_ms": round(read_ms, 4),
                              "kernels_ms_per_step": ks}), flush=True)
    for v in variants:
        st = [s for s, _ in res[v]]
        med = {k: round(statistics.median(ks[k] for _, ks in res[v]), 4) for k in kernels}
        print(json.dumps({"variant": v, "median_ms_per_step": round(statistics.median(st), 4),
                          "min_ms_per_step": round(min(st), 4), "median_kernels_ms": med}), flush=True)


if __name__ == "__main__":
    main()
