#!/usr/bin/env python3
"""Placement probe (round 5): does a slow region belong to the physical memory or to one large
allocation?  The plain read (serverGradient fold, k_reduce_vec, best of 3) of 128-row blocks of
C3's rows (D = 10 M, N = 1024, 41 GB) held three ways: one [N, D] tensor; 8 tensors of 128 rows;
1024 separate row tensors (the reference's N client tensors, read through a row-pointer table).
usage: python tools/probe_alloc.py [mode ...]   (modes: one, blocks, rows; default all, in turn)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from flpytorch_amd import aggregation as ag
    n, d, bs = 1024, 10_000_000, 128
    dev = torch.device("cuda", 0)
    modes = sys.argv[1:] or ["one", "blocks", "rows"]
    out = torch.empty(d, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn, reps=3):
        fn()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(reps):
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            best = min(best, e0.elapsed_time(e1))
        return best
    for mode in modes:
        if mode == "one":
            big = torch.empty((n, d), device=dev)
            blocks = [big[b:b + bs] for b in range(0, n, bs)]
        elif mode == "blocks":
            blocks = [torch.empty((bs, d), device=dev) for _ in range(0, n, bs)]
        else:
            rows = [torch.empty(d, device=dev) for _ in range(n)]
            blocks = [rows[b:b + bs] for b in range(0, n, bs)]
        for i, blk in enumerate(blocks):
            if isinstance(blk, list):
                for r in blk:
                    r.normal_()
            else:
                blk.normal_()
            t = timed(lambda: ag.reduce_rows(out, blk, relative=False, out=out))
            print(json.dumps({"mode": mode, "block": i, "read_ms": round(t, 3),
                              "read_TBps": round(bs * d * 4 / 1e9 / t, 3)}), flush=True)
        del blocks
        if mode == "one":
            del big
        elif mode == "rows":
            del rows
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
