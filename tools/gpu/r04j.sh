#!/bin/bash
# round 4: side-stream TopK selects in 256-thread workgroups (co-resident with the filter) vs 512
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04j}; mkdir -p $out
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_parity.py -k "topk" > $out/tests.log 2>&1 || exit $?
A="python tools/ab_inproc.py --rounds 4 --steps 5 --prof-modes off"
timeout -k 10 400 $A --workload c3 --variants prod,s512 > $out/ab_c3_a.txt 2>&1 || exit $?
timeout -k 10 400 $A --workload c3 --variants s512,prod > $out/ab_c3_b.txt 2>&1 || exit $?
timeout -k 10 400 python tools/ab_inproc.py --rounds 3 --steps 5 --no-bitcheck --workload c3 --variants prod,fp1 > $out/ab_c3_fp.txt 2>&1 || exit $?
exit 0
