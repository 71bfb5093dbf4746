#!/bin/bash
# round 3 (session 3): TopK sample loads in one round trip (16 per thread) — the TopK GPU tests,
# then the lone-row drop-in line against HEAD (alternating processes) and C3 in-process
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03s2ab16; mkdir -p $out
timeout -k 10 400 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread -x tests -m gpu -k "topk or parity or select or dropin" > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $out/tests.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR|E )" $out/tests.log | head -20; exit 1; }
rm -f $out/dropin.log
for rep in 1 2; do
  for v in head prod; do
    vv=$v; [ $v = prod ] && vv=""
    FLC_LIB_VARIANT=$vv timeout -k 10 300 python bench.py --dropin --workload c3 --n 8 --steps 10 --warmup 2 > $out/run.log 2>&1 || { tail -20 $out/run.log; exit 1; }
    echo "$v $(grep '^{' $out/run.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(r["us_per_call"], r["per_kernel_us"])')" >> $out/dropin.log
  done
done
cat $out/dropin.log
timeout -k 10 400 python tools/ab_inproc.py --workload c3 --variants head,prod --rounds 3 > $out/inproc_c3.log 2>&1 || { tail -20 $out/inproc_c3.log; exit 1; }
grep median $out/inproc_c3.log
