#!/bin/bash
# same-box A/B of library variants over several workloads: VARIANTS="head nt" WLS="c4 c3"; each
# variant run twice interleaved per workload; one line per run: wl tag ms_per_step kernel_ms others
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/ab; mkdir -p $out; rm -f $out/ab.log
if [ -n "$TESTS" ]; then   # TESTS="tag@VAR=val:regex": GPU tests of that variant first
  tv=${TESTS%%:*}; rx=${TESTS#*:}; v=${tv%%@*}; ev=""; [ "$tv" != "$v" ] && ev=${tv#*@}
  env $ev FLC_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "$rx" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
  tail -2 $out/tests.log
fi
for wla in ${WLS:-c4 c3}; do
  wl=${wla//+/ }   # "c4+--compat+--n+256": extra bench args joined by +
  for rep in 1 2; do
    for va in ${VARIANTS:-head nt}; do
      v=${va%%@*}; ev=""; [ "$va" != "$v" ] && ev=${va#*@}   # "tuning@FLC_DS_RB=16": variant + one env knob
      [ "$v" = prod ] && v=""                                 # "prod": the product libflcodec.so
      env $ev FLC_LIB_VARIANT=$v timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline $BENCH_ARGS > $out/run.log 2>&1 || exit $?
      echo "$wla $va $(tail -1 $out/run.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r["kernel_ms_per_step"], r.get("other_kernels_avg_ms"))')" >> $out/ab.log
    done
  done
done
cat $out/ab.log
exit 0
