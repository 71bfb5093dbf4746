#!/bin/bash
# Round 6: the drop-in TopK call's floors — load / store of the row (tools/probe_lone_floor.hip) and
# one grid-barrier round (tools/probe_gridbar.hip)
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_floor; mkdir -p $o
timeout -k 10 120 tools/probe_lone_floor 10000000 32 20 0 > $o/floor_default.jsonl 2>&1 && \
timeout -k 10 60 tools/probe_gridbar 245 200 > $o/gridbar.jsonl 2>&1
rc=$?; cat $o/floor_default.jsonl $o/gridbar.jsonl; exit $rc
