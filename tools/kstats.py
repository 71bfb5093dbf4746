"""Print the per-kernel averages of the newest rocprofv3 kernel_stats.csv under a directory."""
import csv
import glob
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_c3"
files = sorted(glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True), key=os.path.getmtime)
for r in csv.DictReader(open(files[-1])):
    print("%-64s %5s %10.1f us" % (r["Name"][:64], r["Calls"], float(r["AverageNs"]) / 1000))
