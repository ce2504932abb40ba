#!/bin/bash
# merge_small_kernel phase shares (stamps build) on C4 (generation and actor-major orders) + a C4 bench line.
set -o pipefail
mkdir -p gpurun_out
HMGPU_LIB=hypermerge_amd/_lib/ablate/lib_stamps_base.so timeout -k 10 200 python tools/stamps.py C4 1000000 > gpurun_out/stamps_c4.log 2>&1 || exit 2
HMGPU_LIB=hypermerge_amd/_lib/ablate/lib_stamps_base.so timeout -k 10 200 python tools/stamps.py C4 1000000 1 > gpurun_out/stamps_c4am.log 2>&1 || exit 2
grep -v amdgpu.ids gpurun_out/stamps_c4.log; grep -v amdgpu.ids gpurun_out/stamps_c4am.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-traffic --no-e2e --no-incremental --no-node > gpurun_out/bench_c4_quick.log 2>&1 || { tail -5 gpurun_out/bench_c4_quick.log; exit 3; }
tail -1 gpurun_out/bench_c4_quick.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C4 value %.4e ms %.3f frac %.4f kernels %s orders %s' % (d['value'], d['ms_per_step'], d['roofline']['frac'], [(k['kernel'], round(k['ms'],3)) for k in d['roofline']['kernels']], d.get('arrival_orders')))"
