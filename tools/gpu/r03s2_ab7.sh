#!/bin/bash
# round 3 (session 2): C4 row groups (the fold of group g under the filter of g + 1) re-measured on
# one allocation with this round's fold; then bench.py's multi-rank paths rehearsed (2 ranks on the
# box's one GPU over gloo: weak C3, fixed-N C4, C5)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03s2ab7; mkdir -p $out
timeout -k 10 500 python tools/ab_inproc.py --workload c4 --variants prod,prod:rg2,prod:rg4 --rounds 3 > $out/inproc_c4_rg.log 2>&1 || { tail -20 $out/inproc_c4_rg.log; exit 1; }
grep median $out/inproc_c4_rg.log
bash tools/gpu/rehearse_dist.sh || exit $?
for f in weak strong c5; do echo "$f: $(grep '^{' gpurun_out/rehearse/$f.log | tail -1 | cut -c1-220)"; done
