#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r06_tnprobe; mkdir -p $o
FLC_LIB_VARIANT=tnprint PYTHONPATH=. timeout -k 10 120 python tools/probe_tn.py > $o/probe.txt 2>&1 || { tail $o/probe.txt; exit 1; }
grep -c "tn part" $o/probe.txt; grep "tn lane" $o/probe.txt; grep "tn part" $o/probe.txt | head -3
