#!/usr/bin/env python3
"""In-process A/B of the lone compressVector (drop-in TopK / QSGD) across library builds (GPU box).

Every variant (abvar/libflcodec_<tag>.so, "prod" = the product library) is loaded into one process
and timed on the same rows, rounds interleaved: mean device time of one compressVector over n rows
(HIP events around calls back to back on the current stream), per variant and round, and the
outputs compared bit for bit against the first variant's.

usage: python tools/ab_lone.py --variants prod,r05 [--spec topk:1%] [--d 10000000] [--n 8] [--rounds 6]
"""
import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="prod,r05")
    ap.add_argument("--spec", default="topk:1%")
    ap.add_argument("--d", type=int, default=10_000_000)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--calls", type=int, default=12, help="passes over the n rows per timing")
    ap.add_argument("--compat", action="store_true", help="dithering: the numpy-stream uniforms (the drop-in's draws)")
    a = ap.parse_args()
    import numpy as np
    from flpytorch_amd import _lib
    from flpytorch_amd import aggregation as ag
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    gen = torch.Generator(device=dev).manual_seed(9)
    rows = torch.randn(a.n, a.d, generator=gen, device=dev)
    comps = [ag.initCompressor(a.spec, a.d) for _ in range(a.n)]
    if a.compat or not a.spec.startswith(("topk", "randk")):
        rs = np.random.RandomState(123)
        for i, c in enumerate(comps):
            c.generateCompressPattern(rs, "cuda", i, {})
            if hasattr(c, "testp") and torch.is_tensor(c.testp):
                c.testp = c.testp.to(dev)
    variants = a.variants.split(",")
    libs = {v: _lib.open_variant(v) for v in variants}
    ref = {}

    def run_all():
        return [comps[i].compressVector(rows[i]) for i in range(a.n)]

    res = {v: [] for v in variants}
    for r in range(a.rounds):
        # the variants' order reversed every other round: no variant always runs first / after another
        for v in (variants if r % 2 == 0 else variants[::-1]):
            with _lib.use(libs[v]):
                outs = run_all()                                   # warm + output for the bit check
                torch.cuda.synchronize()
                if v == variants[0] and r == 0:
                    ref = [o.view(torch.int32).clone() for o in outs]
                else:
                    same = all(torch.equal(o.view(torch.int32), q) for o, q in zip(outs, ref))
                    if not same:
                        print(json.dumps({"variant": v, "round": r, "bits": "DIFFER"}), flush=True)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.calls):
                    for i in range(a.n):
                        comps[i].compressVector(rows[i])
                e1.record()
                e1.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / (a.calls * a.n)
                res[v].append(us)
                print(json.dumps({"variant": v, "round": r, "us_per_call": round(us, 2)}), flush=True)
    for v in variants:
        print(json.dumps({"variant": v, "spec": a.spec, "d": a.d, "median_us_per_call": round(statistics.median(res[v]), 2),
                          "min": round(min(res[v]), 2), "rounds": [round(x, 2) for x in res[v]]}), flush=True)


if __name__ == "__main__":
    main()
