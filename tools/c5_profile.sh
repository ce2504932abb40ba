#!/bin/bash
# C5 evidence (VERDICT r02 "why does C5 run at 4.7 %"): per-kernel split, phase stamps, rocprofv3
# kernel stats and PMC counters for the C5 workload (100k nested map/list documents).
set -o pipefail
OUT=${1:-gpurun_out/c5}
mkdir -p $OUT
timeout -k 10 300 python bench.py --config C5 --docs 100000 --steps 10 --warmup 2 --no-cpu --no-traffic --no-e2e --no-incremental --no-node > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit 1
HMGPU_LIB=hypermerge_amd/_lib/ablate/lib_stamps.so timeout -k 10 200 python tools/stamps.py C5 100000 > $OUT/stamps_c5.log 2>&1 || exit 2
bash tools/profile.sh c5prof --config C5 --docs 100000 > $OUT/profile.log 2>&1 || exit 3
python3 tools/pmc_summary.py gpurun_out/c5prof/pmc1 > $OUT/pmc1.json; python3 tools/pmc_summary.py gpurun_out/c5prof/pmc2 > $OUT/pmc2.json
python3 tools/pmc_summary.py gpurun_out/c5prof/pmc3 > $OUT/pmc3.json; python3 tools/pmc_summary.py gpurun_out/c5prof/pmc4 > $OUT/pmc4.json
cp gpurun_out/c5prof/trace/*kernel_stats.csv $OUT/ 2>/dev/null
echo done
