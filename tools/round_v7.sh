#!/bin/bash
# GPU round: all GPU tests, the default bench line (traffic, e2e, CPU legs), per-config table.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 700 python bench.py > gpurun_out/bench_v7.log 2>&1 || { tail -20 gpurun_out/bench_v7.log; exit 2; }
tail -1 gpurun_out/bench_v7.log
timeout -k 10 1000 python tools/perf_table.py ${1:-C1,C2,C3,C5} > gpurun_out/perf_table.md 2>&1 || { cat gpurun_out/perf_table.md; exit 3; }
grep -v '^<!--' gpurun_out/perf_table.md
