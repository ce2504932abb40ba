#!/bin/bash
# General-kernel iteration round: large-kernel parity tests, then A/B stamps + C3/C1 bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_store_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_res.log 2>&1 || { echo "tests failed"; grep -E "Error|error|assert|FAIL" gpurun_out/gpu_tests_res.log | head -30; tail -30 gpurun_out/gpu_tests_res.log; exit 1; }
tail -2 gpurun_out/gpu_tests_res.log
bash tools/ab_large.sh "$@"
