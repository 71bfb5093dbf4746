#!/bin/bash
# Round 6: k_lone_resident without agent-scope fences (FLC_RS_FENCE=0, write-through hand-offs):
# the lone-row suites on the variant, the per-workgroup timeline, then a same-process A/B
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r06_s30; mkdir -p $o
FLC_LIB_VARIANT=s3 timeout -k 10 600 python -u -m pytest tests/test_gpu_tie.py tests/test_gpu_parity.py tests/test_gpu_rows_ref.py tests/test_gpu_resident.py tests/test_gpu_threads.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
FLC_LIB_VARIANT=rsprint PYTHONPATH=. timeout -k 10 120 python tools/probe_lone_tl.py 10000000 4 > $o/tl.txt 2>&1 || exit 1
grep -E "rs_tl|flags" $o/tl.txt | tail -4
PYTHONPATH=. timeout -k 10 300 python tools/ab_lone.py --variants s2,s3 --n 32 --rounds 6 > $o/ab.jsonl 2>&1 || exit 1
grep -E "median|DIFFER" $o/ab.jsonl
