#!/bin/bash
# GPU round: parity tests, A/B of the queue-emulation change on blocked workloads.
set -o pipefail
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 gpurun_out/gpu_tests.log
for c in ${CFGS:-"C4 1000000" "C5 100000" "C4 1000000 1"}; do
  set -- $c
  for so in hypermerge_amd/_lib/ablate/lib_*.so; do
    a=""; [ -n "$3" ] && a="--arrival $3"
    HMGPU_LIB=$so timeout -k 10 300 python bench.py --config $1 --docs $2 $a --steps 5 --warmup 2 --no-cpu --no-traffic --no-e2e > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 2; }
    echo "$c $(basename $so) $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("ms/step %.3f small %.3f parity %s" % (d["ms_per_step"], d["roofline"]["kernel_ms"], d["parity_sample_ok"]))')"
  done
done
