"""One step's kernel timeline from a rocprofv3 --kernel-trace CSV: every kernel from the last
launch of the step's first kernel (default k_ds_sample) on, start / end in us from that launch.

usage: python tools/timeline.py <dir with *kernel_trace.csv> [first-kernel-substring] [nth-from-last] [launches per step]
"""
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
first = sys.argv[2] if len(sys.argv) > 2 else "k_ds_sample"
nth = int(sys.argv[3]) if len(sys.argv) > 3 else 2
f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True), key=os.path.getmtime)[-1]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
stride = int(sys.argv[4]) if len(sys.argv) > 4 else 1      # launches of the first kernel per step
starts = starts[::stride]
i0 = starts[-nth]
i1 = starts[-nth + 1] if nth > 1 else len(rows)
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i1]:
    nm = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print("%9.1f %9.1f %8.1f  q%-3s %s" % (s / 1e3, e / 1e3, (e - s) / 1e3, r.get("Queue_Id", "?"), nm[:70]))
