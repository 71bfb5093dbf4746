#!/bin/bash
# C4 fold occupancy: k_ds_accum built for 5 / 6 waves per SIMD (w5 / w6: a temporary
# amdgpu_waves_per_eu on the kernel, not kept in the tree) against the product (98 VGPRs: 4)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/awpe; mkdir -p $o
timeout -k 10 600 python3 tools/ab_inproc.py --workload c4 --variants prod,w5,w6 --rounds 3 --steps 5 --prof-modes on > $o/ab.log 2>&1 || { tail -20 $o/ab.log; exit 1; }
tail -3 $o/ab.log
