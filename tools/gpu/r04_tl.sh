#!/bin/bash
# kernel traces of short C4 / C3 bench runs (one step's timeline: tools/timeline.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=$GRAFT_REPO_ROOT/gpurun_out/tl; mkdir -p $o
cd /tmp && export TMPDIR=/tmp
for wl in c4 c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $o/$wl -o tr --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload $wl --steps 4 --warmup 2 --no-cpu-baseline > $o/$wl.log 2>&1 || exit 1
done
cd $GRAFT_REPO_ROOT
python3 tools/timeline.py $o/c4 k_ds_sample 2 > $o/c4_tl.txt
python3 tools/timeline.py $o/c3 k_topk_sample 2 > $o/c3_tl.txt
