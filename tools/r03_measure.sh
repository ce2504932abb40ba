#!/bin/bash
# Round-3 measurement pass: per-config kernel lines, then the C5 evidence (stamps, rocprofv3 stats, PMC).
set -o pipefail
mkdir -p gpurun_out/r03
bash tools/quick_cfg.sh gpurun_out/r03/quick "C4:1000000 C2:100000 C5:100000 C3:10000" > gpurun_out/r03/quick.txt 2>&1 || { cat gpurun_out/r03/quick.txt; exit 1; }
cat gpurun_out/r03/quick.txt
bash tools/c5_profile.sh gpurun_out/r03/c5 > gpurun_out/r03/c5.txt 2>&1 || { cat gpurun_out/r03/c5.txt; exit 2; }
cat gpurun_out/r03/c5/stamps_c5.log | grep -v amdgpu.ids
cat gpurun_out/r03/c5/*kernel_stats.csv | head -8
