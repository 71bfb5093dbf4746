#!/usr/bin/env python3
"""Placement probe (round 6): the C4 shard's rows allocated physically contiguous
(hipExtMallocWithFlags(..., hipDeviceMallocContiguous)) against torch's default allocation, in one
process, rounds alternating: the plain read of every 64-row block (k_reduce_vec) and the C4 step
(qsgd:127 fused encode + reduce).  The slow blocks of a default allocation showed more address
translation misses (profiles/r06/regions_pmc.jsonl); a contiguous allocation maps with the
largest page fragments.  usage: python tools/probe_contig.py [--rounds 3]"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _Dev:
    def __init__(self, ptr, n, d):
        self.__cuda_array_interface__ = {"shape": (n, d), "typestr": "<f4", "data": (ptr, False), "version": 3,
                                         "strides": None}


def contiguous_rows(n, d):
    hip = ctypes.CDLL("libamdhip64.so")
    p = ctypes.c_void_p()
    rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(n * d * 4), ctypes.c_uint(0x4))
    if rc != 0:
        raise RuntimeError(f"hipExtMallocWithFlags(contiguous) failed: {rc}")
    return torch.as_tensor(_Dev(p.value, n, d), device="cuda"), (hip, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    from flpytorch_amd import aggregation as ag
    n, d = 512, 25_000_000
    dev = torch.device("cuda", 0)
    out = torch.empty(d, device=dev)
    rows = {}
    gen = torch.Generator(device=dev).manual_seed(1000)
    rows["default"] = torch.empty((n, d), dtype=torch.float32, device=dev)
    rows["contiguous"], keep = contiguous_rows(n, d)
    for k in rows:
        g = torch.Generator(device=dev).manual_seed(1000)
        for i in range(0, n, 64):
            rows[k][i:i + 64].normal_(generator=g)
    torch.cuda.synchronize()
    red = ag.UplinkReducer(ag.initCompressor("qsgd:127", d), device=dev, seed=20241015)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / reps

    ref = None
    for r in range(a.rounds):
        for k, x in rows.items():
            blocks = [round(64 * d * 4 / 1e9 / timed(lambda b=b: ag.reduce_rows(out, x[b:b + 64], relative=False, out=out), 2), 3)
                      for b in range(0, n, 64)]
            read = timed(lambda: ag.reduce_rows(out, x, relative=False, out=out), 2)
            step = timed(lambda: red(x, out=out), a.steps)
            bits = out.view(torch.int32).clone()
            if ref is None:
                ref = bits
            same = bool(torch.equal(bits, ref))
            print(json.dumps({"round": r, "alloc": k, "block_read_TBps": blocks, "read_ms": round(read, 4),
                              "c4_step_ms": round(step, 4), "same_bits": same}), flush=True)


if __name__ == "__main__":
    main()
