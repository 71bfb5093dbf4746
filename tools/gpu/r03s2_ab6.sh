#!/bin/bash
# round 3 (session 2): C3 tail scheduling — a smaller last row group (its select is the exposed tail)
# and the samples of groups 1.. under group 0's filter: TopK GPU tests of the es125 variant, then an
# in-process A/B (prod = the old schedule through the new code path)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03s2ab6; mkdir -p $out
T="python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 600 $T -x tests -m gpu > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $out/tests.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR|E )" $out/tests.log | head -20; exit 1; }
FLC_LIB_VARIANT=es125 timeout -k 10 600 $T -x tests/test_gpu_parity.py tests/test_gpu_configs.py -k "topk or c3 or fold" > $out/tests_es125.log 2>&1; rc=$?
echo "es125 tests rc=$rc $(tail -1 $out/tests_es125.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR|E )" $out/tests_es125.log | head -20; exit 1; }
timeout -k 10 500 python tools/ab_inproc.py --workload c3 --variants head,prod,l125,l60,es,es125 --rounds 4 > $out/inproc_c3.log 2>&1 || { tail -20 $out/inproc_c3.log; exit 1; }
grep median $out/inproc_c3.log
