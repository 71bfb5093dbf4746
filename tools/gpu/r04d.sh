#!/bin/bash
# round 4: C4 filter probes (outputs invalid; only the filter's time is read), same allocation
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04d}; mkdir -p $out
A="python tools/ab_inproc.py --rounds 3 --steps 4 --no-bitcheck"
timeout -k 10 400 $A --workload c4 --variants prod,p6,p3 > $out/ab_c4_probe.txt 2>&1 || exit $?
exit 0
