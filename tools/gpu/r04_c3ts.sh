#!/bin/bash
# C3: the number of TopK row groups (FLC_ROW_GROUPS hint; the exposed last group fold tile: CHUNK measured best) (same allocation, in-process A/B, bit-checked)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/c3ts; mkdir -p $o
timeout -k 10 600 python3 tools/ab_inproc.py --workload c3 --variants prod,prod:rg3,prod:rg6,prod:rg8 --rounds 5 --steps 5 --prof-modes off > $o/ab.log 2>&1 || { tail -20 $o/ab.log; exit 1; }
tail -15 $o/ab.log
