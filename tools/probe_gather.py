#!/usr/bin/env python3
"""Calibration probe (not product code): HBM cost of sparse 4-B gathers, the access pattern of the
RandK gather (x[S] at ~1 % density).  A 4 GiB fp32 buffer, sorted random index sets at a few
densities, torch index_select timed with events; run it under `rocprofv3 --pmc FETCH_SIZE` (and a
separate pass for TCC_EA0_RDREQ_sum) to see how many bytes a touched sector costs.

usage: python tools/probe_gather.py [--reps 5]
"""
import argparse
import json

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    n = 1 << 30
    x = torch.empty(n, dtype=torch.float32, device="cuda").normal_()
    g = torch.Generator(device="cuda").manual_seed(3)
    for dens in (1.0 / 64, 0.01, 0.002):
        k = int(n * dens)
        idx = torch.randperm(n, generator=g, device="cuda")[:k].sort().values
        out = torch.empty(k, dtype=torch.float32, device="cuda")
        torch.index_select(x, 0, idx, out=out)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            torch.index_select(x, 0, idx, out=out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        res = {"density": dens, "k": k, "ms": round(ms, 4), "elements_per_s": k / ms * 1e3}
        for sec in (32, 64, 128):
            per = sec // 4
            touched = n / per * (1.0 - (1.0 - dens) ** per)
            res[f"sector{sec}_GBps"] = round(touched * sec / ms / 1e6, 1)
        res["idx_bytes"] = k * 8
        print(json.dumps(res), flush=True)
        del idx, out


if __name__ == "__main__":
    main()
