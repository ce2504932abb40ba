#!/bin/bash
# Round-6 incremental-round breakdown: C4 (1M docs) per-phase log + kernel stats; C5 (100k docs)
# incremental mode 1 vs re-merge only, per-phase logs and kernel stats.
set -o pipefail
OUT=gpurun_out/${1:-r06/incprof}
R=$PWD
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/inc_round.sh ${1:-r06/incprof}/c4 nopmc || exit 1
for M in 1 0; do
  timeout -k 10 200 python tools/inc_profile.py --config C5 --docs 100000 --device 1 --incremental $M > $OUT/c5_m$M.log 2>&1 || exit 2
  cd /tmp
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/c5_m$M -o run -- python3 $R/tools/inc_profile.py --config C5 --docs 100000 --device 1 --incremental $M > $R/$OUT/c5_m${M}_trace.log 2>&1 || exit 3
  cd $R
done
for M in 1 0; do echo "== C5 mode $M"; grep -v amdgpu $OUT/c5_m$M.log | tail -12; f=$(find $OUT/c5_m$M -name "*kernel_stats.csv" | head -1); head -14 $f | cut -d, -f1-5; done
