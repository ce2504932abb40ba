#!/bin/bash
# C5 resident rounds (100k documents), incremental mode 1 vs re-merge only: kernel stats of each
# (rocprofv3 --kernel-trace --stats).  tools/c5_modes.sh <out>
set -o pipefail
OUT=gpurun_out/${1:-c5modes}
R=$PWD
mkdir -p $OUT
export TMPDIR=/tmp
for M in 1 0; do
  cd /tmp
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/c5_m$M -o run -- python3 $R/tools/inc_profile.py --config C5 --docs 100000 --device 1 --incremental $M > $R/$OUT/c5_m${M}_trace.log 2>&1 || exit 3
  cd $R
done
for M in 1 0; do echo "== C5 mode $M"; grep -v amdgpu $OUT/c5_m${M}_trace.log | tail -6; f=$(find $OUT/c5_m$M -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | cut -c1-150 | head -24; done
