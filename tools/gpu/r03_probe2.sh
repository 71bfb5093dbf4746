#!/bin/bash
# round 3: where the C4 filter's time goes (tuning build probes; outputs not valid): 0 full,
# 2 no candidate staging, 3 loads + norm only, 4 group hash without multiplies
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03p2; mkdir -p $out
VARIANTS="tuning@FLC_DS_PROBE=0 tuning@FLC_DS_PROBE=2 tuning@FLC_DS_PROBE=3 tuning@FLC_DS_PROBE=4 g1" WLS="c4" bash tools/gpu/ab_wl.sh > $out/ab_stdout.log 2>&1 || exit $?
cp gpurun_out/ab/ab.log $out/ab.log
cat $out/ab.log
exit 0
