#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r06_contig; mkdir -p $o
timeout -k 10 300 python tools/probe_contig.py --rounds 3 > $o/contig.jsonl 2> $o/contig.err || { tail -5 $o/contig.err; exit 1; }
cat $o/contig.jsonl
