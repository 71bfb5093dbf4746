#!/bin/bash
# Round 6: placement diagnosis of the C4 shard's slow rows.  Plain-read timing
# of every 64-row block under four allocation layouts, then PMC passes (translation, L2 / EA,
# latency) per block of the bench's single-allocation layout (tools/probe_regions.py).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r06_regions
mkdir -p $out
timeout -k 10 300 python tools/probe_regions.py --reps 3 > $out/timing.jsonl 2> $out/timing.err || exit $?
timeout -k 10 300 python tools/probe_regions.py --reps 3 --modes split32,halves,big,single > $out/timing_rev.jsonl 2> $out/timing_rev.err || exit $?
P1="TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_STALL_MULTI_MISS_sum"
P2="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum"
P3="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum"
P4="TCC_EA0_RDREQ_LEVEL_sum TCC_BUSY_sum TCC_HIT_sum TCC_MISS_sum"
P5="TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY"
i=0
for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $out/pmc$i -o run --output-format csv -- \
     python3 tools/probe_regions.py --modes single,halves --reps 1 > $out/pmc$i.log 2>&1 || exit $?
done
exit 0
