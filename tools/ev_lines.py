"""Summarise an evidence pass's bench lines: python tools/ev_lines.py gpurun_out/<ev>"""
import glob
import json
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "*.log"))):
    lines = [l for l in open(f, errors="replace") if l.startswith("{")]
    if not lines:
        continue
    try:
        j = json.loads(lines[-1])
    except ValueError:
        continue
    r = j.get("roofline") or {}
    print(f"{os.path.basename(f):28s} value={j.get('value')} ms={j.get('ms_per_step')} pct={j.get('pct_hbm_peak')} "
          f"kern={r.get('kernel')} frac={r.get('frac')} avg={r.get('avg_launch_ms')} read={r.get('read_ceiling_GBps')} "
          f"fr_read={r.get('frac_of_read_ceiling')} us_call={r.get('us_per_call')} others={r.get('other_kernels_avg_ms') or r.get('per_kernel_us')}")
