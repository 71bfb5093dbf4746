#!/bin/bash
# round 4: QSGD row groups (whole tail on the side stream) x filter LDS pad (5 / 4 blocks per CU)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04l}; mkdir -p $out
A="python tools/ab_inproc.py --rounds 3 --steps 5 --prof-modes off"
timeout -k 10 500 $A --workload c4 --variants prod,pad5k:rg2,pad5k:rg3,pad10k:rg2,pad10k:rg3 > $out/ab_c4_rg_a.txt 2>&1 || exit $?
timeout -k 10 500 $A --workload c4 --variants pad5k:rg3,pad5k:rg2,prod,pad10k:rg3,pad10k:rg2 > $out/ab_c4_rg_b.txt 2>&1 || exit $?
exit 0
