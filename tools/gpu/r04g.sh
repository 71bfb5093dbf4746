#!/bin/bash
# round 4: does the bench's kernel timing (a hipEvent pair around every hot launch) slow the step?
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04g}; mkdir -p $out
A="python tools/ab_inproc.py --rounds 4 --steps 5 --prof-modes on,off"
timeout -k 10 400 $A --workload c3 --variants prod > $out/ab_c3.txt 2>&1 || exit $?
timeout -k 10 400 $A --workload c4 --variants prod > $out/ab_c4.txt 2>&1 || exit $?
exit 0
