#!/bin/bash
# Round 6: the speculative round with an 8-bit second digit (b8: 3 x 256 window bins, a 19-bit
# prefix of up to RS_CAP candidates) vs the full 11-bit digit (b11)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r06_b8; mkdir -p $o
FLC_LIB_VARIANT=b8 timeout -k 10 600 python -u -m pytest tests/test_gpu_tie.py tests/test_gpu_parity.py tests/test_gpu_rows_ref.py tests/test_gpu_resident.py tests/test_gpu_threads.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
PYTHONPATH=. timeout -k 10 300 python tools/ab_lone.py --variants b11,b8 --n 32 --rounds 6 > $o/ab.jsonl 2>&1 || exit 1
grep -E "median|DIFFER" $o/ab.jsonl
