#!/bin/bash
# One drop-in compressVector call's kernel timeline (rocprofv3 --kernel-trace) and the bench line.
#   usage: tools/gpu/dropin_tl.sh <out-tag> [workload c3|c4] [variant]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
root=$GRAFT_REPO_ROOT; tag=$1; wl=${2:-c3}; v=${3:-}
o=$root/gpurun_out/$tag; mkdir -p $o
first=$([ "$wl" = c3 ] && echo k_topk_sample || echo k_norm_partials)
cd /tmp && export TMPDIR=/tmp
FLC_LIB_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace -d $o/trd_$wl -o tr --output-format csv -- \
    python3 $root/bench.py --dropin --workload $wl --n 8 --steps 10 --warmup 2 > $o/dropin_$wl${v:+_$v}.log 2>&1 || exit 1
cd $root
{ echo "== dropin $wl $v"; python3 tools/timeline.py $o/trd_$wl $first 3; } >> $o/dropin_tl.txt
rm -rf $o/trd_$wl
FLC_LIB_VARIANT=$v timeout -k 10 300 python3 bench.py --dropin --workload $wl --n 8 --steps 20 --warmup 3 > $o/dropin_plain_$wl${v:+_$v}.log 2>&1 || exit 1
cat $o/dropin_tl.txt
