#!/bin/bash
# Round 6: k_lone_resident with fewer VALU ops per row element (v1: window histogram, candidate
# count / list / dense tests; v2: + the ranking workgroup ranks before its dense stores) vs cur
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r06_dn; mkdir -p $o
FLC_LIB_VARIANT=dn timeout -k 10 600 python -u -m pytest tests/test_gpu_tie.py tests/test_gpu_parity.py tests/test_gpu_rows_ref.py tests/test_gpu_resident.py tests/test_gpu_threads.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
PYTHONPATH=. timeout -k 10 300 python tools/ab_lone.py --variants dn0,dn --n 32 --rounds 6 > $o/ab.jsonl 2>&1 || exit 1
grep -E "median|DIFFER" $o/ab.jsonl
