#!/bin/bash
# round 3 (session 2): all GPU tests, then in-process A/Bs (one allocation): C3 with the 5-wave
# whole-chunk TopK fold (prod) against 4-wave blocks (ca4) and the previous build (head); C4 head vs prod
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03s2ab4; mkdir -p $out
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread -x tests -m gpu > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $out/tests.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR|E )" $out/tests.log | head -20; exit 1; }
timeout -k 10 400 python tools/ab_inproc.py --workload c3 --variants head,prod,ca4 --rounds 4 > $out/inproc_c3.log 2>&1 || { tail -20 $out/inproc_c3.log; exit 1; }
timeout -k 10 400 python tools/ab_inproc.py --workload c4 --variants head,prod --rounds 3 > $out/inproc_c4.log 2>&1 || { tail -20 $out/inproc_c4.log; exit 1; }
timeout -k 10 400 python tools/ab_inproc.py --workload c2 --variants head,prod --rounds 3 > $out/inproc_c2.log 2>&1 || { tail -20 $out/inproc_c2.log; exit 1; }
tail -3 $out/inproc_c3.log; tail -2 $out/inproc_c4.log; tail -2 $out/inproc_c2.log
