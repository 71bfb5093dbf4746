#!/usr/bin/env python3
"""Placement probe (round 5): the plain read (serverGradient fold, k_reduce_vec) of each 64-row block
of the C4 shard's resident [512, 25 M] allocation, best of 3, so a slow physical region of the
allocation shows up as slow blocks.  Also the same blocks through the QSGD filter (one fused call of
64 rows each)."""
import json
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from flpytorch_amd import aggregation as ag
    n, d = 512, 25_000_000
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(1000)
    rows = torch.empty((n, d), dtype=torch.float32, device=dev)
    for i in range(0, n, 64):
        rows[i:i + 64].normal_(generator=gen)
    out = torch.empty(d, device=dev)
    red = ag.UplinkReducer(ag.initCompressor("qsgd:127", d), device=dev, seed=20241015)
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
    res = []
    for b in range(0, n, 64):
        blk = rows[b:b + 64]
        t_read = timed(lambda: ag.reduce_rows(out, blk, relative=False, out=out))
        t_qsgd = timed(lambda: red(blk, out=out))
        gb = 64 * d * 4 / 1e9
        res.append({"rows": [b, b + 64], "read_ms": round(t_read, 3), "read_TBps": round(gb / t_read, 3),
                    "qsgd_ms": round(t_qsgd, 3), "qsgd_TBps": round(gb / t_qsgd, 3),
                    "addr_GB": round((rows[b].data_ptr() - rows.data_ptr()) / 1e9, 1)})
        print(json.dumps(res[-1]), flush=True)


if __name__ == "__main__":
    main()
