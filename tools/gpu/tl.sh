#!/bin/bash
# One step's kernel timeline (rocprofv3 --kernel-trace + tools/timeline.py) per case.
#   usage: tools/gpu/tl.sh <out-tag> <workload> <case>...
#   case = <variant>[:rg<K>][@VAR=VAL[,VAR=VAL...]]   (variant "prod" = product .so; VARs for tuning builds)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
root=$GRAFT_REPO_ROOT; tag=$1; wl=$2; shift 2
o=$root/gpurun_out/$tag; mkdir -p $o
first=$([ "$wl" = c3 ] && echo k_topk_sample || echo k_ds_sample)
for cs in "$@"; do
  base=${cs%%@*}; envs=""; [[ $cs == *@* ]] && envs=${cs#*@}
  v=${base%%:*}; rg=""; [[ $base == *:rg* ]] && rg="--row-groups ${base##*:rg}"
  ve=""; [ "$v" != prod ] && ve=$v
  name=$(echo "$cs" | tr '@,=:' '____')
  cd /tmp && export TMPDIR=/tmp
  env FLC_LIB_VARIANT=$ve ${envs//,/ } true || exit 1
  ( export FLC_LIB_VARIANT=$ve; for kv in ${envs//,/ }; do export "$kv"; done
    timeout -k 10 300 rocprofv3 --kernel-trace -d $o/tr_$name -o tr --output-format csv -- \
      python3 $root/bench.py --workload $wl --steps 4 --warmup 2 --no-cpu-baseline $rg > $o/bench_$name.log 2>&1 ) || exit 1
  cd $root
  { echo "== $cs"; grep -h '^{' $o/bench_$name.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('ms_per_step', d['ms_per_step'])"; \
    python3 tools/timeline.py $o/tr_$name $first 2 $([ "$wl" = c3 ] || [ "$wl" = c4 ] && echo 2 || echo 1); } >> $o/tl_$wl.txt
  rm -rf $o/tr_$name
done
cat $o/tl_$wl.txt
