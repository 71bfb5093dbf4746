#!/bin/bash
# round 3 (session 2), verdict item 2: the round-1 TopK filter build (git a21cf89, its own bench.py
# in abtree_r01/) against the current build on C3, alternating fresh processes on one box
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03s2r01; mkdir -p $out; rm -f $out/lines.jsonl
for rep in 1 2 3; do
  for t in r01 cur; do
    if [ $t = r01 ]; then b=abtree_r01/bench.py; else b=bench.py; fi
    timeout -k 10 300 python $b --steps 10 --warmup 2 --no-cpu-baseline > $out/run.log 2>&1 || { tail -20 $out/run.log; exit 1; }
    echo "{\"tree\": \"$t\", \"rep\": $rep, \"line\": $(tail -1 $out/run.log)}" >> $out/lines.jsonl
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r03s2r01/lines.jsonl"):
    d = json.loads(l); r = d["line"]; rf = r["roofline"]
    print(d["tree"], d["rep"], r["ms_per_step"], rf.get("kernel_ms_per_step", rf.get("kernel_ms")), rf.get("read_ceiling_GBps"))
PY
exit 0
