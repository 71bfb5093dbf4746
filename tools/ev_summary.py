"""Print the numbers DESIGN.md's evidence table quotes from one evidence directory
(profiles/r03/<dir>/, made by tools/collect_final.sh).   usage: python tools/ev_summary.py profiles/r03/final"""
import csv
import json
import os
import sys

d = sys.argv[1]


def line(name):
    p = os.path.join(d, name + ".jsonl")
    return json.load(open(p)) if os.path.exists(p) else None


def rocprof_avg_us(wl, kernel):
    p = os.path.join(d, f"{wl}_kernel_stats.csv")
    if not os.path.exists(p):
        return None
    for r in csv.DictReader(open(p)):
        if kernel in r["Name"]:
            return round(float(r["AverageNs"]) / 1e3, 1)
    return None


print(open(os.path.join(d, "BUILD.txt")).read().strip())
print("tests:", open(os.path.join(d, "gpu_tests_summary.txt")).read().strip())
for name in ["bench_default", "bench_c3", "bench_c4", "bench_c4_plain", "bench_c4_strong", "bench_c4_compat", "bench_c5",
             "bench_c2", "bench_reduce"]:
    j = line(name)
    if not j:
        continue
    r = j["roofline"]
    wl = name.split("_")[1] if name.count("_") == 1 else None
    rp = rocprof_avg_us(wl, r.get("kernel", "")) if wl in ("c2", "c3", "c4", "c5") else None
    print(f"{name}: {j['ms_per_step']} ms  {j['value']} {j['unit']}  kernel={r.get('kernel')} "
          f"kernel_ms={r.get('kernel_ms_per_step')} achieved={r['achieved']} frac={r['frac']} "
          f"read_ceiling={r.get('read_ceiling_GBps')} frac_rc={r.get('frac_of_read_ceiling')} rocprof_us={rp} "
          f"others={r.get('other_kernels_avg_ms')}")
for name in ["dropin_c3", "dropin_c4"]:
    j = line(name)
    if j:
        r = j["roofline"]
        print(f"{name}: {r.get('us_per_call')} us/call frac={r['frac']} per_kernel={r.get('per_kernel_us')}")
for wl in ("c2", "c3", "c4"):
    p = os.path.join(d, f"pmc_{wl}.json")
    if os.path.exists(p):
        j = json.load(open(p))
        print(f"pmc {wl}: {j['kernel']} {j['hbm_bytes_per_launch'] / 1e9:.3f} GB/launch")
