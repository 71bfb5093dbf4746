#!/bin/bash
# Same-allocation A/B of library builds (tools/ab_inproc.py) on the GPU box.
#   usage: tools/gpu/ab.sh <out-tag> <workload> <variants> [rounds] [extra ab_inproc args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
tag=$1; wl=$2; vars=$3; rounds=${4:-3}; shift 4 2>/dev/null || shift $#
o=gpurun_out/$tag; mkdir -p $o
timeout -k 10 900 python3 -u tools/ab_inproc.py --workload $wl --variants $vars --rounds $rounds --steps 5 "$@" > $o/ab_$wl.log 2>&1 || { tail -20 $o/ab_$wl.log; exit 1; }
grep median $o/ab_$wl.log
