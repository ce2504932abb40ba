#!/bin/bash
# Kernel-variant round: parity tests (default build), per-phase PMC + kernel_ms of the ablation builds.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_store_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash tools/phase_pmc.sh || exit 2
timeout -k 10 600 python tools/ablate.py hypermerge_amd/_lib/ablate/lib_a*.so || exit 3
