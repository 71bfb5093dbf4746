#!/bin/bash
# round 3 (session 3): QSGD sample of 64K elements on 1024 threads (tighter norm bounds: fewer
# candidates and ambiguous entries) — the QSGD GPU tests, then C4 in-process A/B against HEAD's
# 16K sample and a 1 % margin variant
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03s2ab15; mkdir -p $out
timeout -k 10 400 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread -x tests -m gpu -k "dither or qsgd or parity" > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $out/tests.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR|E )" $out/tests.log | head -20; exit 1; }
timeout -k 10 500 python tools/ab_inproc.py --workload c4 --variants head,prod,m1 --rounds 4 > $out/inproc_c4.log 2>&1 || { tail -20 $out/inproc_c4.log; exit 1; }
grep median $out/inproc_c4.log
