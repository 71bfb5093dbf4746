#!/usr/bin/env python3
"""Per-block PMC counters of tools/probe_regions.py (--reps 1) from rocprofv3 --pmc passes: the
k_reduce_vec dispatches in order are [warm, block 0..7] per layout; prints one line per block with
every pass's counters beside the block's plain-read rate from the same pass's log.
usage: python tools/probe_regions_pmc.py gpurun_out/r06_regions"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    rows = defaultdict(dict)         # (layout index, block) -> counters
    rates = {}
    for p in sorted(glob.glob(os.path.join(root, "pmc*"))):
        if not os.path.isdir(p):
            continue
        f = glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True)
        if not f:
            continue
        disp = defaultdict(dict)
        with open(f[0]) as fh:
            for r in csv.DictReader(fh):
                if "k_reduce_vec" not in r["Kernel_Name"]:
                    continue
                disp[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        ids = sorted(disp)
        # per layout: a warm dispatch then 8 blocks
        for li in range(len(ids) // 9):
            for b in range(8):
                rows[(li, b)].update(disp[ids[li * 9 + 1 + b]])
        log = p + ".log"
        if os.path.exists(log):
            for line in open(log):
                if line.startswith("{"):
                    d = json.loads(line)
                    rates.setdefault((d["mode"], d["block"]), []).append(d["TBps"])
    modes = ["single", "halves"]
    for (li, b), c in sorted(rows.items()):
        m = modes[li] if li < len(modes) else str(li)
        r = rates.get((m, b), [])
        keys = sorted(c)
        print(json.dumps({"mode": m, "block": b, "TBps_per_pass": r, **{k: c[k] for k in keys}}))


if __name__ == "__main__":
    main()
