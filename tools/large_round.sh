#!/bin/bash
# merge_large_kernel iteration round (via gpurun): parity tests, phase shares (stamps build), C3/C1 bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
if [ -f hypermerge_amd/_lib/ablate/lib_stamps.so ]; then
  HMGPU_LIB=hypermerge_amd/_lib/ablate/lib_stamps.so timeout -k 10 200 python tools/lstamps.py C3 10000 > gpurun_out/lstamps_c3.log 2>&1 || exit 2
  cat gpurun_out/lstamps_c3.log
fi
for cd in ${CONFIGS:-C3:10000}; do
  c=${cd%%:*}; nd=${cd##*:}
  timeout -k 10 300 python bench.py --config $c --docs $nd --check-docs 200 --steps 5 --warmup 2 --no-cpu --no-traffic > gpurun_out/bench_$c.log 2>&1 || { tail -5 gpurun_out/bench_$c.log; exit 3; }
  tail -1 gpurun_out/bench_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c value %.3e  ms %.3f parity %s unsup %s' % (d['value'], d['ms_per_step'], d['parity_sample_ok'], d['unsupported_docs']))"
done
