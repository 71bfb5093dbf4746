#!/bin/bash
# round 3 (session 2): few-row TopK candidate select with every digit in one launch (k_cs_all) —
# all GPU tests, then the drop-in line against csm (one k_cs_pass launch per digit), alternating
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03s2ab9; mkdir -p $out
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread -x tests -m gpu > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $out/tests.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR|E )" $out/tests.log | head -20; exit 1; }
rm -f $out/dropin.log
for rep in 1 2; do
  for v in csm prod; do
    vv=$v; [ $v = prod ] && vv=""
    FLC_LIB_VARIANT=$vv timeout -k 10 300 python bench.py --dropin --workload c3 --n 8 --steps 10 --warmup 2 > $out/run.log 2>&1 || { tail -20 $out/run.log; exit 1; }
    echo "$v $(grep '^{' $out/run.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(r["us_per_call"], r["per_kernel_us"])')" >> $out/dropin.log
  done
done
cat $out/dropin.log
