#!/bin/bash
# Round 6: per-workgroup timelines of back-to-back lone TopK calls, two stamp sets (FLC_RS_PRINT builds)
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_tl2; mkdir -p $o
for v in rsA rsB; do
  FLC_LIB_VARIANT=$v PYTHONPATH=. timeout -k 10 120 python tools/probe_lone_tl.py 10000000 4 > $o/$v.txt 2>&1 || exit 1
  echo $v; grep -E "rs_tl" $o/$v.txt | tail -3
done
