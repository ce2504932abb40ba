#!/bin/bash
# round 4: the C5 resident rounds under rocprofv3 (kernel stats) and the store's phase marks
set -o pipefail
O=gpurun_out/r04/${1:-c5inc}
R=$PWD
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python tools/inc_profile.py --config C5 --docs 100000 --device 1 > $O/phases.log 2>&1 || { tail -20 $O/phases.log; exit 1; }
grep -v amdgpu.ids $O/phases.log | tail -40
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o run -- python3 $R/tools/inc_profile.py --config C5 --docs 100000 --device 1 > $R/$O/trace.log 2>&1 || exit 2
cd $R
f=$(find $O/trace -name "*kernel_stats.csv" | head -1); cut -c1-150 $f | head -16
