#!/bin/bash
cd "$GRAFT_REPO_ROOT"
G="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_INSTS_VALU_INT32,SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_LDS,SQ_INSTS_LDS,SQ_LEVEL_WAVES SQ_THREAD_CYCLES_VALU,SQ_BUSY_CYCLES,GRBM_GUI_ACTIVE,SQ_INST_LEVEL_VMEM"
tools/pmc_passes.sh c4 --workload c4 --n 64 --steps 1 --warmup 0 -- $G || exit $?
tools/pmc_passes.sh red --workload reduce --n 64 --steps 1 --warmup 0 -- $G || exit $?
exit 0
