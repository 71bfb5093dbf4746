#!/bin/bash
# round 3 (session 2): one-wave fold workgroups (sparse-QSGD fold with a per-row ring, TopK chunk
# fold with its -0 masks in the workspace) — all GPU tests, a same-box A/B against the previous
# build (head) on C4 and C3, then the filter probes and SQ counters (tools/gpu/r03s2_probe.sh)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03s2f; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $out/tests.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR|E )" $out/tests.log | head -20; exit 1; }
VARIANTS="head prod" WLS="c4 c3" bash tools/gpu/ab_wl.sh > $out/ab_stdout.log 2>&1 || exit $?
cp gpurun_out/ab/ab.log $out/ab.log
cat $out/ab.log
VARIANTS="prod" WLS="c4+--row-groups+2 c4+--row-groups+4 c4+--row-groups+8" bash tools/gpu/ab_wl.sh > $out/ab_stdout.log 2>&1 || exit $?
cp gpurun_out/ab/ab.log $out/ab_rg.log
cat $out/ab_rg.log
bash tools/gpu/r03s2_probe.sh
