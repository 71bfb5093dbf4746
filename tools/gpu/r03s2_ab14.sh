#!/bin/bash
# round 3 (session 2): the TopK filter's candidate test as one float compare (!(|x| < T)) — all GPU
# tests, then C3 in-process A/B against icmp (the and + integer compare)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03s2ab14; mkdir -p $out
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread -x tests -m gpu > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $out/tests.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR|E )" $out/tests.log | head -20; exit 1; }
timeout -k 10 400 python tools/ab_inproc.py --workload c3 --variants icmp,prod --rounds 5 > $out/inproc_c3.log 2>&1 || { tail -20 $out/inproc_c3.log; exit 1; }
grep median $out/inproc_c3.log
