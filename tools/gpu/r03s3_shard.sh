#!/bin/bash
# round 3 (session 3): few-row shards keyed by the group's index within its row (the fused n <= 16
# uplink overflowed its shards) + ties resolved by k_cs_pass — all GPU tests, drop-in lines under
# rocprofv3, C3 in-process against HEAD (the many-row path must be unchanged)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03s3shard; mkdir -p $out
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread -x tests -m gpu > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $out/tests.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR|E )" $out/tests.log | head -20; exit 1; }
bash tools/gpu/dropin_prof.sh || exit 1
timeout -k 10 400 python tools/ab_inproc.py --workload c3 --variants head,prod --rounds 3 > $out/inproc_c3.log 2>&1 || { tail -20 $out/inproc_c3.log; exit 1; }
grep median $out/inproc_c3.log
