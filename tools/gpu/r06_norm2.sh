#!/bin/bash
# Round 6: the torch-order norm in parallel (binade-segment maps) — parity tests and the drop-in price
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r06_norm2; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_norm_torch.py tests/test_gpu_rows_ref.py -x -q -p no:cacheprovider \
   --timeout 200 --timeout-method thread -rf > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 300 python bench.py --dropin --workload c4 --n 4 --steps 3 --warmup 1 --norm-mode torch_cpu > $o/dropin_c4_torchnorm.log 2>&1 || exit 1
tail -1 $o/dropin_c4_torchnorm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['us_per_call'], d['roofline']['per_kernel_us'])"
