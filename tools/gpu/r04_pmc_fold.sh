#!/bin/bash
# fold kernels' address-translation and cache counters (C3 and C4, one step each)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/pmcf; mkdir -p $o
timeout -s KILL 60 rocprofv3 -L > $o/list.txt 2>&1
grep -o "TCP_UTCL1[A-Z_]*\|UTCL2[A-Z_]*\|TCP_TCC_READ_REQ_sum\|TCP_PENDING_STALL_CYCLES_sum" $o/list.txt | sort -u > $o/avail.txt
cat $o/avail.txt | head -20
P1=$(grep -x "TCP_UTCL1_TRANSLATION_MISS_sum\|TCP_UTCL1_TRANSLATION_HIT_sum\|TCP_TCC_READ_REQ_sum\|TCP_PENDING_STALL_CYCLES_sum" $o/avail.txt | tr '\n' ' ')
[ -z "$P1" ] && { echo "no TCP counters"; exit 0; }
for wl in c3 c4; do
  timeout -s KILL 90 rocprofv3 --pmc $P1 -d $o/$wl -o run --output-format csv -- python3 bench.py --workload $wl --steps 1 --warmup 0 --no-cpu-baseline > $o/$wl.log 2>&1 || exit 1
done
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $o/c4h -o run --output-format csv -- python3 bench.py --workload c4 --steps 1 --warmup 0 --no-cpu-baseline > $o/c4h.log 2>&1 || exit 1
exit 0
