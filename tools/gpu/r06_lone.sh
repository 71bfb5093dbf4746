#!/bin/bash
# Round 6: the resident lone-TopK abort + repair: its GPU tests, then an
# in-process A/B of the clean path's cost against the round-5 build (abvar/libflcodec_r05.so).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r06_lone
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tie.py tests/test_gpu_threads.py -x -q -p no:cacheprovider \
   --timeout 120 --timeout-method thread -rf > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python tools/ab_lone.py --variants prod,nof,r05 --rounds 8 > $out/ab_lone_topk.jsonl 2>&1 || exit 1
tail -2 $out/ab_lone_topk.jsonl
exit 0
