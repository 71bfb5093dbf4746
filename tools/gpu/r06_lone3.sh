#!/bin/bash
# Round 6: where a lone TopK call's time goes now (printf phase stamps, FLC_RS_PRINT build) and the
# lazy completion event (FLC_RS_EVREC=0) A/B
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r06_lone3; mkdir -p $o
FLC_LIB_VARIANT=rsprint PYTHONPATH=. timeout -k 10 120 python tools/probe_lone.py 10000000 6 > $o/stamps.txt 2>&1 || exit 1
grep -E "rs_stamps|rs_skew|flags" $o/stamps.txt | tail -6
timeout -k 10 300 python tools/ab_lone.py --variants prod,ev0,r05 --rounds 10 > $o/ab.jsonl 2>&1 || exit 1
grep median $o/ab.jsonl
