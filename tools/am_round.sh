#!/bin/bash
# queue-history round: small-kernel parity (queue orders, duplicates, cycles), C4 actor-major stamps, quick C4 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_am.log 2>&1 || { echo "tests failed"; grep -E "^(FAILED|ERROR)" gpurun_out/gpu_tests_am.log | head; tail -20 gpurun_out/gpu_tests_am.log; exit 1; }
tail -1 gpurun_out/gpu_tests_am.log
HMGPU_LIB=hypermerge_amd/_lib/ablate/lib_stamps_base.so timeout -k 10 200 python tools/stamps.py C4 1000000 1 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --no-traffic --no-e2e --no-incremental --no-node > gpurun_out/bench_c4_quick.log 2>&1 || { tail -5 gpurun_out/bench_c4_quick.log; exit 3; }
tail -1 gpurun_out/bench_c4_quick.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C4 value %.4e ms %.3f frac %.4f actor-major %.4e (%.3f ms)' % (d['value'], d['ms_per_step'], d['roofline']['frac'], d['arrival_orders']['actor_major']['value'], d['arrival_orders']['actor_major']['ms_per_step']))"
