#!/bin/bash
# round 4: the C5 (100k) and C4 (1M) resident rounds' append census (HM_STORE_PROFILE), phase
# marks, and the C5 rounds' store kernels under rocprofv3
set -o pipefail
O=gpurun_out/r04/census
R=$PWD
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python tools/inc_profile.py --config C5 --docs 100000 --device 1 --incremental 0 > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
timeout -k 10 240 python tools/inc_profile.py --config C4 --docs 1000000 --device 1 --incremental 0 > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 1; }
grep -h "append\|round" $O/c5.log $O/c4.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o run -- python3 $R/tools/inc_profile.py --config C5 --docs 100000 --device 1 --incremental 0 > $R/$O/trace.log 2>&1 || exit 2
cd $R
f=$(find $O/trace -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | cut -c1-110 | head -12
