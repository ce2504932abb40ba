#!/bin/bash
# targeted GPU tests (argument: pytest -k expression), then stop
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "$1" > gpurun_out/t_quick.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/t_quick.log | head -40; tail -5 gpurun_out/t_quick.log; exit 1; }
tail -3 gpurun_out/t_quick.log
