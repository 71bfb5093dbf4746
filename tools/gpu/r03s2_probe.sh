#!/bin/bash
# round 3 (session 2): where the C4 filter's time goes on one box — tuning-build probes (outputs of
# 2/3 are not valid: 2 no candidate staging, 3 loads + norm only, 5 exec-narrowed staging without
# a branch) interleaved with the full filter, then SQ counters of the product's C4 kernels
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r03s2p; mkdir -p $out
VARIANTS="tuning@FLC_DS_PROBE=0 tuning@FLC_DS_PROBE=2 tuning@FLC_DS_PROBE=3 tuning@FLC_DS_PROBE=5" WLS="c4" bash tools/gpu/ab_wl.sh > $out/ab_stdout.log 2>&1 || exit $?
cp gpurun_out/ab/ab.log $out/ab.log
G1="SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_VMEM"
G2="SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_BRANCH,SQ_WAIT_ANY,SQ_LEVEL_WAVES,SQ_INSTS_VMEM_RD,SQ_IFETCH"
G3="GRBM_GUI_ACTIVE,SQ_WAVES,SQ_INSTS_SMEM,SQ_INST_LEVEL_VMEM,SQ_LDS_BANK_CONFLICT,SQ_INSTS_VMEM_WR"
tools/pmc_passes.sh c4sq --workload c4 --steps 1 --warmup 0 -- $G1 $G2 $G3 || exit $?
for k in k_ds_filter k_ds_accum k_ds_resolve; do
  echo "== $k"; python tools/pmc_summary.py $k $(find gpurun_out/pmc_c4sq_* -name "*counter_collection.csv")
done > $out/sq.txt
cat $out/ab.log
exit 0
