#!/bin/bash
# One GPU verification round (run via gpurun from the repo root): parity tests, stamp shares,
# bench.  Each GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
if [ -f hypermerge_amd/_lib/ablate/lib_stamps.so ]; then
  HMGPU_LIB=hypermerge_amd/_lib/ablate/lib_stamps.so timeout -k 10 300 python tools/stamps.py C4 1000000 > gpurun_out/stamps_c4.log 2>&1 || exit 2
  HMGPU_LIB=hypermerge_amd/_lib/ablate/lib_stamps.so timeout -k 10 300 python tools/stamps.py C2 100000 > gpurun_out/stamps_c2.log 2>&1 || exit 3
  cat gpurun_out/stamps_c4.log gpurun_out/stamps_c2.log
fi
timeout -k 10 300 python bench.py --no-cpu --steps 20 > gpurun_out/bench.log 2>&1 || exit 4
tail -1 gpurun_out/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.3e  kernel_ms %.3f  frac %.3f parity %s' % (d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['parity_sample_ok']))"
