#!/bin/bash
# round 4: TopK row-group folds (select + exact fallback in one workgroup, each group's fold under the
# next group's filter) and the C4 2-group default: GPU suite, then same-allocation A/Bs
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04m}; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || exit $?
A="python tools/ab_inproc.py --rounds 4 --steps 5 --prof-modes off"
timeout -k 10 400 $A --workload c3 --variants prod,ngf > $out/ab_c3.txt 2>&1 || exit $?
timeout -k 10 400 $A --workload c4 --variants prod,prod:rg1 > $out/ab_c4.txt 2>&1 || exit $?
timeout -k 10 400 $A --workload c3 --variants ngf,prod > $out/ab_c3_b.txt 2>&1 || exit $?
exit 0
