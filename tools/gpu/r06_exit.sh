#!/bin/bash
# Round 6: k_lone_resident cut short (cost probes): the loads only (ex1), + the sample's digit (ex2)
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_exit; mkdir -p $o
PYTHONPATH=. timeout -k 10 300 python tools/ab_lone.py --variants s2,ex1,ex2,ex3 --n 32 --rounds 4 > $o/ab.jsonl 2>&1
rc=$?; grep -E "median" $o/ab.jsonl; exit $rc
