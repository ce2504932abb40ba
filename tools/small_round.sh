#!/bin/bash
# merge_small_kernel iteration round (via gpurun): parity tests, then bench lines per config:docs[:arrival].
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for spec in ${CONFIGS:-C4:1000000}; do
  IFS=: read c nd arr <<< "$spec"
  extra=""; [ -n "$arr" ] && extra="--arrival $arr"
  timeout -k 10 300 python bench.py --config $c --docs $nd --check-docs 2000 --steps 10 --warmup 2 --no-cpu --no-traffic --no-e2e $extra > gpurun_out/bench_$c$arr.log 2>&1 || { tail -5 gpurun_out/bench_$c$arr.log; exit 3; }
  tail -1 gpurun_out/bench_$c$arr.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$spec value %.3e  ms %.3f kernel_ms %.3f unsup %s' % (d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['unsupported_docs']))"
done
