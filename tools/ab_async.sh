#!/bin/bash
# A/B of the small kernel's async next-row loads (tools/build_variants.sh libs), C4 both orders + C2
set -o pipefail
O=gpurun_out/${1:-ab_async}
mkdir -p $O
L=hypermerge_amd/_lib/ablate
for rep in 1 2; do
  timeout -k 10 300 python tools/ablate.py $L/lib_base.so $L/lib_async.so >> $O/c4.log 2>&1 || exit 1
done
ABL_ARGS="--arrival 1" timeout -k 10 300 python tools/ablate.py $L/lib_base.so $L/lib_async.so >> $O/c4am.log 2>&1 || exit 2
ABL_CONFIG=C2 ABL_DOCS=100000 timeout -k 10 300 python tools/ablate.py $L/lib_base.so $L/lib_async.so >> $O/c2.log 2>&1 || exit 3
cat $O/c4.log $O/c4am.log $O/c2.log
