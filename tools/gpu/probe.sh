#!/bin/bash
# MALL-reuse probe + SQ counters of the C4 encode kernel
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 tools/probe_mall 64 25000000 > gpurun_out/probe_mall.log 2>&1 || exit $?
timeout -k 10 120 tools/probe_mall 64 10000000 >> gpurun_out/probe_mall.log 2>&1 || exit $?
G="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_LDS,SQ_BUSY_CYCLES,GRBM_GUI_ACTIVE"
tools/pmc_passes.sh c4 --workload c4 --n 64 --steps 1 --warmup 0 -- $G || exit $?
exit 0
