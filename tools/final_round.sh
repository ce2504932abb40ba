#!/bin/bash
# Round-end measurement: default bench line (traffic, e2e, CPU legs), rocprofv3 kernel trace +
# PMC passes of the same workload, and the per-config table.  Usage: tools/final_round.sh <tag>
set -o pipefail
TAG=${1:-final}
mkdir -p gpurun_out
timeout -k 10 700 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
bash tools/profile.sh $TAG || exit 2
python tools/pmc_summary.py gpurun_out/$TAG > gpurun_out/$TAG/pmc_summary.json || exit 3
timeout -k 10 1000 python tools/perf_table.py > gpurun_out/perf_table_$TAG.md 2>&1 || { cat gpurun_out/perf_table_$TAG.md; exit 4; }
grep -v '^<!--' gpurun_out/perf_table_$TAG.md
