#!/bin/bash
# GPU tests against an A/B variant build (FLC_LIB_VARIANT=<tag>): usage tools/gpu/varianttests.sh <out-tag> <variant> <pytest args...>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
tag=$1; v=$2; shift 2
o=gpurun_out/$tag; mkdir -p $o
FLC_LIB_VARIANT=$v timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread "$@" > $o/tests_$v.log 2>&1; rc=$?
tail -3 $o/tests_$v.log
exit $rc
