#!/bin/bash
# Round 6: per-group exit counters — the forced-abort tests and the lone A/B against round 5
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r06_b2; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_tie.py tests/test_gpu_threads.py -x -q -p no:cacheprovider \
   --timeout 120 --timeout-method thread -rf > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 300 python tools/ab_lone.py --variants prod,nof,nocnt --rounds 8 > $o/ab1.jsonl 2>&1 || exit 1
timeout -k 10 300 python tools/ab_lone.py --variants r05,prod --rounds 8 > $o/ab2.jsonl 2>&1 || exit 1
grep median $o/ab*.jsonl
