#!/bin/bash
# the bench lines over fresh allocations on one box: each run is its own process (its own placement
# of the rows); WLS="c4 c3", RUNS=3.  One JSON line per run in gpurun_out/alloc_median/<wl>.jsonl
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/alloc_median; mkdir -p $out
for wl in ${WLS:-c4 c3}; do
  rm -f $out/$wl.jsonl
  for i in $(seq ${RUNS:-3}); do
    timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline > $out/run.log 2>&1 || { tail -20 $out/run.log; exit 1; }
    grep '^{' $out/run.log | tail -1 >> $out/$wl.jsonl
  done
  python - $out/$wl.jsonl <<'PY'
import json, statistics, sys
L = [json.loads(x) for x in open(sys.argv[1])]
ms = [d["ms_per_step"] for d in L]; k = [d["roofline"]["kernel_ms_per_step"] for d in L]
rc = [d["roofline"]["read_ceiling_GBps"] for d in L]
print(sys.argv[1].split("/")[-1], "ms", ms, "median", statistics.median(ms), "kernel", k, "read_ceiling", rc)
PY
done
