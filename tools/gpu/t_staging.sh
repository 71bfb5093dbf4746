#!/bin/bash
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; out=gpurun_out/ts; mkdir -p $out
FLC_LIB_VARIANT=buggy timeout -k 10 300 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "staging_capacity" > $out/buggy.log 2>&1
tail -3 $out/buggy.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
