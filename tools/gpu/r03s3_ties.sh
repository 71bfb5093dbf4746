#!/bin/bash
# round 3 (session 3): few-row TopK with ambiguous ties at the K-th key resolved by k_cs_pass's last
# arriver (was: the 8 ms exact path) — the TopK GPU tests, then the drop-in lines under rocprofv3
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03s3ties; mkdir -p $out
timeout -k 10 400 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread -x tests -m gpu -k "topk or parity or select or dropin or limits" > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $out/tests.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR|E )" $out/tests.log | head -20; exit 1; }
bash tools/gpu/dropin_prof.sh
