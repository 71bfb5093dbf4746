#!/usr/bin/env python3
"""Sum rocprofv3 counter CSVs per kernel-name substring: pmc_summary.py <kernel-substr> <csv>..."""
import collections
import csv
import sys

sub = sys.argv[1]
agg = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in sys.argv[2:]:
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
for k in sorted(agg):
    print(f"{k:32s} {agg[k]:18.0f}  dispatches={len(disp[k])}")
