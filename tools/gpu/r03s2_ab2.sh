#!/bin/bash
# round 3 (session 2): GPU tests of the product (one-wave XCD-mapped TopK fold, sparse-QSGD fold
# ring) and of the ILP filter variant, then in-process A/Bs on one allocation (tools/ab_inproc.py),
# then the round-1 vs current C3 A/B (verdict item 2)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03s2ab2; mkdir -p $out
T="python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 600 $T -x tests -m gpu > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $out/tests.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR|E )" $out/tests.log | head -20; exit 1; }
FLC_LIB_VARIANT=ilp timeout -k 10 600 $T -x tests/test_gpu_dither_sparse.py tests/test_gpu_configs.py > $out/tests_ilp.log 2>&1; rc=$?
echo "ilp tests rc=$rc $(tail -1 $out/tests_ilp.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR|E )" $out/tests_ilp.log | head -20; exit 1; }
timeout -k 10 400 python tools/ab_inproc.py --workload c4 --variants head,prod,ilp --rounds 5 > $out/inproc_c4.log 2>&1 || { tail -20 $out/inproc_c4.log; exit 1; }
timeout -k 10 400 python tools/ab_inproc.py --workload c3 --variants head,prod,ca4 --rounds 5 > $out/inproc_c3.log 2>&1 || { tail -20 $out/inproc_c3.log; exit 1; }
tail -3 $out/inproc_c4.log; tail -3 $out/inproc_c3.log
bash tools/gpu/r03s2_r01ab.sh
