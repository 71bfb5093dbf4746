#!/bin/bash
# TopK lone row: k_cs_pass list mode (two launches) vs head (three); TopK parity first
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/lone_ab; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rows_ref.py -x -q --timeout 120 --timeout-method thread -k "topk or TopK or few" > $o/tests_topk.log 2>&1 || { tail -30 $o/tests_topk.log; exit 1; }
tail -1 $o/tests_topk.log
for rep in 1 2; do
for v in prod head nolist; do
  if [ $v = prod ]; then unset FLC_LIB_VARIANT; else export FLC_LIB_VARIANT=$v; fi
  timeout -k 10 120 python3 tools/dropin_probe.py > $o/t_$v.json || exit 1
  echo "$rep topk $v $(cat $o/t_$v.json)"
done
done
unset FLC_LIB_VARIANT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$o/prof -o tr -- python3 $GRAFT_REPO_ROOT/tools/dropin_probe.py --reps 40 > $GRAFT_REPO_ROOT/$o/prof.log 2>&1
