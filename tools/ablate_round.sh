#!/bin/bash
# GPU round for kernel variants: parity tests on the default build, then kernel_ms of each
# hypermerge_amd/_lib/ablate/lib_*.so (tools/ablate.py), plus stamp shares if present.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_store_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 600 python tools/ablate.py $(ls hypermerge_amd/_lib/ablate/lib_*.so | grep -v stamps) > gpurun_out/ablate.log 2>&1 || exit 2
cat gpurun_out/ablate.log
if [ -f hypermerge_amd/_lib/ablate/lib_stamps.so ]; then
  HMGPU_LIB=hypermerge_amd/_lib/ablate/lib_stamps.so timeout -k 10 300 python tools/stamps.py C4 1000000 > gpurun_out/stamps_c4.log 2>&1 || exit 3
  cat gpurun_out/stamps_c4.log
fi
