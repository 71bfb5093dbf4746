#!/bin/bash
# One step's kernel timeline (rocprofv3 --kernel-trace + tools/timeline.py) per case.
#   usage: tools/gpu/tl.sh <out-tag> <workload> <case>...   case = <variant>[:rg<K>] (variant "prod" = product .so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
root=$GRAFT_REPO_ROOT; tag=$1; wl=$2; shift 2
o=$root/gpurun_out/$tag; mkdir -p $o
first=$([ "$wl" = c3 ] && echo k_topk_sample || echo k_ds_sample)
for cs in "$@"; do
  v=${cs%%:*}; rg=""; [[ $cs == *:rg* ]] && rg="--row-groups ${cs##*:rg}"
  ve=""; [ "$v" != prod ] && ve=$v
  cd /tmp && export TMPDIR=/tmp
  FLC_LIB_VARIANT=$ve timeout -k 10 300 rocprofv3 --kernel-trace -d $o/tr_$cs -o tr --output-format csv -- \
      python3 $root/bench.py --workload $wl --steps 4 --warmup 2 --no-cpu-baseline $rg > $o/bench_$cs.log 2>&1 || exit 1
  cd $root
  { echo "== $cs"; grep -h '^{' $o/bench_$cs.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('ms_per_step', d['ms_per_step'])"; \
    python3 tools/timeline.py $o/tr_$cs $first 2; } >> $o/tl_$wl.txt
  rm -rf $o/tr_$cs
done
cat $o/tl_$wl.txt
