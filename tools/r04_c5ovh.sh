#!/bin/bash
# round 4: the C5 resident rounds with the incremental path on (mode 1) and off, phase marks and
# kernel stats of each: where mode 1 spends its time over the plain re-merge
set -o pipefail
O=gpurun_out/r04/c5ovh
R=$PWD
mkdir -p $O
export TMPDIR=/tmp
for m in 1 0; do
  timeout -k 10 240 python tools/inc_profile.py --config C5 --docs 100000 --device 1 --incremental $m > $O/phases_$m.log 2>&1 || { tail -20 $O/phases_$m.log; exit 1; }
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace$m -o run -- python3 $R/tools/inc_profile.py --config C5 --docs 100000 --device 1 --incremental $m > $R/$O/trace_$m.log 2>&1 || exit 2
  cd $R
  f=$(find $O/trace$m -name "*kernel_stats.csv" | head -1); echo "== mode $m"; cut -d, -f1-4 $f | cut -c1-120 | head -14
done
grep -h "hm_store\|round" $O/phases_1.log | head -20
grep -h "hm_store\|round" $O/phases_0.log | head -20
