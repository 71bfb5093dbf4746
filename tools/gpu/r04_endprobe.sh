#!/bin/bash
# k_ds_accum end-of-fold cost probes (outputs not valid): e1 without the -0 pass, e2 also without the division
# (the FLC_DS_PROBE_END switch of these probe builds was a temporary patch of k_ds_accum, not kept in the tree:
#  1 = the untouched-column pass skipped, 2 = also out = tile without the division by w_total)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/endp; mkdir -p $o
timeout -k 10 600 python3 tools/ab_inproc.py --workload c4 --variants prod,e1,e2 --rounds 3 --steps 5 --prof-modes on --no-bitcheck > $o/ab.log 2>&1 || { tail -20 $o/ab.log; exit 1; }
tail -3 $o/ab.log
