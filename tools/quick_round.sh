#!/bin/bash
# Full -m gpu suite, then a short C4 bench line (both kernels' times, roofline fraction).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_quick.log 2>&1 || { echo "tests failed"; grep -E "^(FAILED|ERROR)|Error" gpurun_out/gpu_tests_quick.log | head -20; tail -30 gpurun_out/gpu_tests_quick.log; exit 1; }
tail -1 gpurun_out/gpu_tests_quick.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --no-traffic --no-e2e --no-incremental --no-node > gpurun_out/bench_c4_quick.log 2>&1 || { tail -5 gpurun_out/bench_c4_quick.log; exit 3; }
tail -1 gpurun_out/bench_c4_quick.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C4 value %.4e ms %.3f frac %.4f kernels %s actor-major %.4e' % (d['value'], d['ms_per_step'], d['roofline']['frac'], [(k['kernel'], round(k['ms'],3)) for k in d['roofline']['kernels']], d['arrival_orders']['actor_major']['value']))"
