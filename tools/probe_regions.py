#!/usr/bin/env python3
"""Placement diagnosis (round 6): why the C4 shard's rows past ~32 GB of one
allocation read ~10 % slower.  The plain read (serverGradient fold, k_reduce_vec) of each 64-row
block (6.4 GB) of the bench's [512, 25 M] rows, under several allocation layouts, so that a
layout-relative effect (offset inside an allocation) can be told from a physical one (which memory
the driver handed out):

  single    one [512, D] tensor (the bench's layout)
  halves    two [256, D] tensors (25.6 GB each, both below the 32 GB mark)
  big       one [640, D] tensor (64 GB), the first 512 rows used
  split32   two [320, D] tensors (32 GB each), the first 256 rows of each used

Every block is one k_reduce_vec dispatch per repetition, in block order, so that a rocprofv3
--pmc pass attributes counters to blocks by dispatch order (tools/probe_regions_pmc.py).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def layout(mode, n, d, dev, gen):
    if mode == "single":
        t = [torch.empty((n, d), dtype=torch.float32, device=dev)]
        blocks = [t[0][b:b + 64] for b in range(0, n, 64)]
    elif mode == "halves":
        t = [torch.empty((n // 2, d), dtype=torch.float32, device=dev) for _ in range(2)]
        blocks = [x[b:b + 64] for x in t for b in range(0, n // 2, 64)]
    elif mode == "big":
        t = [torch.empty((n + 128, d), dtype=torch.float32, device=dev)]
        blocks = [t[0][b:b + 64] for b in range(0, n, 64)]
    elif mode == "split32":
        t = [torch.empty((320, d), dtype=torch.float32, device=dev) for _ in range(2)]
        blocks = [x[b:b + 64] for x in t for b in range(0, n // 2, 64)]
    else:
        raise SystemExit(mode)
    for x in t:
        for i in range(0, x.shape[0], 64):
            x[i:i + 64].normal_(generator=gen)
    return t, blocks


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="single,halves,big,split32")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--d", type=int, default=25_000_000)
    args = ap.parse_args()
    from flpytorch_amd import aggregation as ag
    dev = torch.device("cuda", 0)
    out = torch.empty(args.d, device=dev)
    for mode in args.modes.split(","):
        gen = torch.Generator(device=dev).manual_seed(1000)
        tensors, blocks = layout(mode, args.n, args.d, dev, gen)
        base = min(x.data_ptr() for x in tensors)
        ag.reduce_rows(out, blocks[0], relative=False, out=out)
        torch.cuda.synchronize()
        res = []
        for bi, blk in enumerate(blocks):
            ts = []
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ag.reduce_rows(out, blk, relative=False, out=out)
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            gb = blk.numel() * 4 / 1e9
            owner = next(i for i, x in enumerate(tensors)
                         if x.data_ptr() <= blk.data_ptr() < x.data_ptr() + x.numel() * 4)
            r = {"mode": mode, "block": bi, "tensor": owner,
                 "offset_in_alloc_GB": round((blk.data_ptr() - tensors[owner].data_ptr()) / 1e9, 1),
                 "va_from_lowest_GB": round((blk.data_ptr() - base) / 1e9, 1),
                 "best_ms": round(min(ts), 3), "TBps": round(gb / min(ts), 3),
                 "all_ms": [round(t, 3) for t in ts]}
            res.append(r)
            print(json.dumps(r), flush=True)
        del tensors, blocks
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
