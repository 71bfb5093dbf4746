#!/bin/bash
# Lone compressVector (drop-in TopK) A/B on one box: per case the plain bench line's us_per_call,
# then (last: a profiler crash ends the script) a kernel timeline of one call per traced case.
#   usage: tools/gpu/lone_ab.sh <tag> "<variant>:<case>" ... [-- "<variant>:<case>:<first kernel>" ...(traced)]
#   case = KEY=VAL env knobs joined by ',' (tuning builds read FLC_* knobs), or "-"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
root=$GRAFT_REPO_ROOT; tag=$1; shift
o=$root/gpurun_out/$tag; mkdir -p $o
export TMPDIR=/tmp
trace=0
for vc in "$@"; do
  [ "$vc" = "--" ] && { trace=1; continue; }
  v=${vc%%:*}; cs=${vc#*:}; first=k_topk_sample
  [ $trace = 1 ] && { first=${cs#*:}; cs=${cs%%:*}; }
  envs=(); [ "$cs" != "-" ] && IFS=',' read -ra envs <<< "$cs"
  if [ $trace = 0 ]; then
    env "${envs[@]}" FLC_LIB_VARIANT=$v timeout -k 10 300 python3 bench.py --dropin --workload c3 --n 8 --steps 20 --warmup 3 > $o/plain_${v}_$cs.log 2>&1 || exit 1
    python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']; print(sys.argv[2], 'us_per_call', r['us_per_call'], r.get('per_kernel_us'))" $o/plain_${v}_$cs.log "$v:$cs" >> $o/lone_ab.txt
  else
    ( cd /tmp && env "${envs[@]}" FLC_LIB_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace -d $o/tr -o tr --output-format csv -- \
        python3 $root/bench.py --dropin --workload c3 --n 8 --steps 10 --warmup 2 > $o/tl_${v}_$cs.log 2>&1 ) || exit 1
    { echo "== $v $cs"; python3 tools/timeline.py $o/tr $first 3; } >> $o/lone_ab.txt
    rm -rf $o/tr
  fi
done
cat $o/lone_ab.txt
