#!/bin/bash
# k_ds_filter cost breakdown on the tuning build (FLC_DS_PROBE: 1 fp32 norm, 2 no staging, 3 loads+norm;
# outputs of probe runs are NOT valid), beside the plain streaming read (reduce)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/dsp; mkdir -p $out; rm -f $out/probe.log
timeout -k 10 300 python bench.py --workload reduce --steps 10 --warmup 2 --no-cpu-baseline > $out/reduce.log 2>&1 || exit $?
echo "reduce $(tail -1 $out/reduce.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')" >> $out/probe.log
for p in ${PROBES:-0 1 2 3 0}; do
  FLC_LIB_VARIANT=tuning FLC_DS_PROBE=$p timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > $out/run.log 2>&1 || exit $?
  echo "$p $(tail -1 $out/run.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r["kernel_ms_per_step"], r.get("other_kernels_avg_ms"))')" >> $out/probe.log
done
exit 0
