#!/bin/bash
# General-kernel measurement round (via gpurun): C3 bench line, phase shares (stamps build),
# rocprofv3 trace + SQ/FETCH/WRITE PMC of C3.  Usage: tools/c3_round.sh <tag>
set -o pipefail
TAG=${1:-c3}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config C3 --docs 10000 --check-docs 200 --steps 5 --warmup 2 --no-cpu --no-traffic > gpurun_out/bench_c3_$TAG.log 2>&1 || { tail -5 gpurun_out/bench_c3_$TAG.log; exit 3; }
tail -1 gpurun_out/bench_c3_$TAG.log
if [ -f hypermerge_amd/_lib/ablate/lib_stamps.so ]; then
  HMGPU_LIB=hypermerge_amd/_lib/ablate/lib_stamps.so timeout -k 10 200 python tools/lstamps.py C3 10000 > gpurun_out/lstamps_c3_$TAG.log 2>&1 || exit 2
  cat gpurun_out/lstamps_c3_$TAG.log
fi
bash tools/profile.sh c3_$TAG --config C3 --docs 10000 || exit 4
python tools/pmc_summary.py gpurun_out/c3_$TAG merge_large_kernel > gpurun_out/c3_$TAG/pmc_summary.json || exit 5
cat gpurun_out/c3_$TAG/pmc_summary.json
