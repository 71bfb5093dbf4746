#!/bin/bash
# Round 6: the sample histogram's LDS replicas (s3: 8) vs one (sr1), same process, rounds alternating
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_sr; mkdir -p $o
PYTHONPATH=. timeout -k 10 300 python tools/ab_lone.py --variants s3,sr1 --n 32 --rounds 8 > $o/ab.jsonl 2>&1 || exit 1
grep -E "median|DIFFER" $o/ab.jsonl
