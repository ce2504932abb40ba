#!/bin/bash
# Bench (full default run, with CPU baseline) + rocprofv3 kernel trace and PMC passes.
# Usage (via gpurun): bash tools/profile_round.sh <tag>
set -o pipefail
TAG=${1:-prof}
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
bash tools/profile.sh $TAG || exit 2
python tools/pmc_summary.py gpurun_out/$TAG > gpurun_out/$TAG/pmc_summary.json || exit 3
cat gpurun_out/$TAG/pmc_summary.json
