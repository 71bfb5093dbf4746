#!/bin/bash
# Round 6: per-workgroup timeline of back-to-back lone TopK calls (FLC_RS_PRINT build)
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_tl; mkdir -p $o
FLC_LIB_VARIANT=rsprint PYTHONPATH=. timeout -k 10 120 python tools/probe_lone_tl.py 10000000 4 > $o/tl.txt 2>&1
rc=$?; grep -E "rs_tl|flags" $o/tl.txt | tail -5; exit $rc
