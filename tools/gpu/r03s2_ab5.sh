#!/bin/bash
# round 3 (session 2): TopK fold in the tail row groups (each group's fold on the side stream after
# its select, under the next group's filter; tiles carried) — all GPU tests, then in-process A/B on
# C3: head (71fb15b), nofov (one fold at the end), prod (4 groups), tg8 (8 groups)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03s2ab5; mkdir -p $out
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread -x tests -m gpu > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $out/tests.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR|E )" $out/tests.log | head -20; exit 1; }
timeout -k 10 500 python tools/ab_inproc.py --workload c3 --variants head,nofov,prod,tg8 --rounds 4 > $out/inproc_c3.log 2>&1 || { tail -20 $out/inproc_c3.log; exit 1; }
grep median $out/inproc_c3.log
