#!/bin/bash
# resident-store round phases (host marks) + kernel stats for incremental and re-merge rounds
set -o pipefail
OUT=gpurun_out/r03/store
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/store_profile.py --rounds 3 --incremental 1 > $OUT/inc.log 2>&1 || { tail -20 $OUT/inc.log; exit 1; }
timeout -k 10 300 python tools/store_profile.py --rounds 3 --incremental 0 > $OUT/remerge.log 2>&1 || { tail -20 $OUT/remerge.log; exit 2; }
R=$PWD
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/trace -o run -- python3 $R/tools/store_profile.py --rounds 3 --incremental 1 > $R/$OUT/trace.log 2>&1 || exit 3
cd $R
grep -v amdgpu.ids $OUT/inc.log | tail -40
grep -v amdgpu.ids $OUT/remerge.log | tail -25
head -14 $OUT/trace/*/run_kernel_stats.csv 2>/dev/null || find $OUT/trace -name "*kernel_stats.csv" -exec head -14 {} \;
