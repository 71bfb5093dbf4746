#!/bin/bash
# A/B: working-tree build vs libflcodec_base.so, interleaved (A B A B) on one box.
# usage: ./gpu_ab.sh <workload> [steps]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
wl=${1:-c3}; steps=${2:-10}
rm -f gpurun_out/ab_$wl.log
for rep in 1 2; do for v in new base; do
  if [ $v = base ]; then export FLC_LIB_VARIANT=base; else unset FLC_LIB_VARIANT; fi
  timeout -k 10 300 python bench.py --workload $wl --steps $steps --warmup 2 --no-cpu-baseline > gpurun_out/ab_run.log 2>&1 || exit $?
  echo "$v $(tail -1 gpurun_out/ab_run.log)" >> gpurun_out/ab_$wl.log
done; done
