#!/bin/bash
# round 4: TopK copy-out in 16-B quads: TopK / RandK / wire GPU tests, then same-allocation A/Bs
# (C3: prod vs the 4-B copy-out; C4: prod vs the pipelined-classification filter)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04f}; mkdir -p $out
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_rows_ref.py tests/test_gpu_shift.py tests/test_gpu_wire.py tests/test_gpu_harness.py -k "topk or c3 or top or harness" > $out/tests.log 2>&1 || exit $?
A="python tools/ab_inproc.py --rounds 4 --steps 4"
timeout -k 10 400 $A --workload c3 --variants prod,cp8 > $out/ab_c3.txt 2>&1 || exit $?
timeout -k 10 400 $A --workload c4 --variants prod,v2 > $out/ab_c4.txt 2>&1 || exit $?
exit 0
