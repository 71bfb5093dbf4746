#!/bin/bash
# Round 6: where k_lone_resident's time goes between the row landing and the first arrival —
# instruction fetch (a ~100 KB kernel run once per launch) vs LDS: PMC passes over lone calls
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r06_pmc_lone; mkdir -p $o
export FLC_LIB_VARIANT=slots0 PYTHONPATH=.
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES" "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAVES" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU"; do
  timeout -k 10 120 rocprofv3 --pmc $grp -d $o/p$i -o run --output-format csv -- python tools/probe_lone_tl.py 10000000 1 > $o/p$i.log 2>&1 || { tail -5 $o/p$i.log; exit 1; }
  i=$((i+1))
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/r06_pmc_lone/p*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "k_lone_resident" in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f.split("/")[2], {k: round(sum(v) / len(v)) for k, v in acc.items()}, "dispatch-rows", {k: len(v) for k, v in acc.items()})
PY
