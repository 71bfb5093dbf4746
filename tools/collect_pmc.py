#!/usr/bin/env python3
"""HBM traffic of the bench's dominant kernel from rocprofv3 PMC counters (run on the GPU box).

Two separate passes (FETCH_SIZE and WRITE_SIZE cannot share one: MI355X_MICROARCH.md "rocprofv3
PMC slots"), each `rocprofv3 --pmc <ctr> -- python bench.py --workload <wl> ...`, then:

    hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 / launches

FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts exactly half the bytes of a wide
(16 B/lane) coalesced streaming read, hence the factor 2 (MI355X_MICROARCH.md §HBM,
cdna_hip_programming.md §7).  Writes to profiles/pmc_<wl>.json, which bench.py reads into
roofline.traffic.

usage: python tools/collect_pmc.py --workload c3 [--n N] [--steps 2]
       python tools/collect_pmc.py --dropin --workload c3 --n 8     (one compressVector: profiles/pmc_dropin_c3.json)
"""
import argparse
import collections
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL_SUBSTR = {"c3": "k_topk_filter_fast", "c4": "k_ds_filter", "reduce": "k_reduce_vec",
                 "c2": "k_randk_gen", "c5": "k_ds_filter"}


DROPIN_KERNEL = {"c3": "k_lone_resident", "c4": "k_lone_dither"}


def run_pass(ctr, wl, extra, outdir, kernel):
    cmd = ["rocprofv3", "--pmc", ctr, "-d", outdir, "-o", "run", "--output-format", "csv", "--",
           sys.executable, os.path.join(ROOT, "bench.py"), "--workload", wl] + extra
    subprocess.run(cmd, check=True, cwd=ROOT, stdout=subprocess.DEVNULL, timeout=600)
    vals, disp = collections.defaultdict(float), set()
    for f in glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                vals[r["Counter_Name"]] += float(r["Counter_Value"])
                disp.add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    return vals[ctr], len(disp)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--kernel", default=None, help="another kernel of the workload (default: its dominant one)")
    ap.add_argument("--tag", default=None, help="output name profiles/pmc_<tag>.json (default: the workload)")
    ap.add_argument("--compat", action="store_true", help="the compat-pattern line (resident numpy-stream patterns)")
    ap.add_argument("--dropin", action="store_true", help="the drop-in line's compressVector kernel")
    a = ap.parse_args()
    kernel = a.kernel or (DROPIN_KERNEL if a.dropin else KERNEL_SUBSTR)[a.workload]
    tag = a.tag or (("dropin_" if a.dropin else "") + a.workload + ("_compat" if a.compat else ""))
    extra = ["--steps", str(a.steps), "--warmup", "1"] + (["--n", str(a.n)] if a.n else []) + (["--compat"] if a.compat else [])
    extra += ["--dropin"] if a.dropin else ["--no-cpu-baseline", "--no-strong-c4"]
    os.environ.setdefault("TMPDIR", "/tmp")
    base = os.path.join(ROOT, "gpurun_out", f"pmc_traffic_{tag}")
    fetch, nf = run_pass("FETCH_SIZE", a.workload, extra, base + "_fetch", kernel)
    write, nw = run_pass("WRITE_SIZE", a.workload, extra, base + "_write", kernel)
    launches = max(nf, nw, 1)
    # what the counters were taken on, so that bench.py attaches them only to a line of the same
    # shape: rows per GPU, D, the dominant kernel's launches per step (the bench
    # runs warmup + the timed steps + the same steps again for the kernel events; a drop-in run
    # launches its kernel once per compressVector)
    sys.path.insert(0, ROOT)
    import bench
    wl = bench.WORKLOADS[a.workload]
    n_rows = a.n or (8 if a.dropin else wl["n"])
    runs = 1 + 2 * a.steps
    res = {"workload": a.workload, "kernel": kernel, "n_override": a.n, "compat": bool(a.compat), "dropin": bool(a.dropin),
           "n": n_rows, "d": wl["d"], "steps": a.steps, "warmup": 1,
           "launches_per_step": None if a.dropin else round(launches / runs, 3),
           "rows_per_launch": 1 if a.dropin else round(n_rows * runs / launches, 3),
           "launches": launches, "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write,
           "hbm_bytes_per_launch": int((2 * fetch + write) * 1024 / launches),
           "correction": "2 x FETCH_SIZE (gfx950 tallies each 128-B line request at 64 B: every streamed "
                         "array here is read as whole lines) + WRITE_SIZE, KiB->B"}
    for d in ("profiles", "gpurun_out"):       # gpurun_out/ is what travels back from the GPU box
        os.makedirs(os.path.join(ROOT, d), exist_ok=True)
        with open(os.path.join(ROOT, d, f"pmc_{tag}.json"), "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
