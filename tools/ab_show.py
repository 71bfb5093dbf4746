"""Summarise gpurun_out/ab_<wl>.log (lines '<variant> <bench json>')."""
import json
import sys

wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
for line in open(f"gpurun_out/ab_{wl}.log"):
    tag, js = line.split(" ", 1)
    d = json.loads(js)
    r = d["roofline"]
    print(f"{tag:5s} value {d['value']:9.1f} {d['unit']}  step {d['ms_per_step']:7.3f} ms  "
          f"{r['kernel']} {r['avg_launch_ms']:7.3f} ms {r['achieved']:7.1f} GB/s")
