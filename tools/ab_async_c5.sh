#!/bin/bash
# A/B of the async next-row loads on the list launches (C5) and C4
set -o pipefail
O=gpurun_out/${1:-ab_async_c5}
mkdir -p $O
L=hypermerge_amd/_lib/ablate
for rep in 1 2; do
  ABL_CONFIG=C5 ABL_DOCS=100000 timeout -k 10 300 python tools/ablate.py $L/lib_base.so $L/lib_a2.so $L/lib_a3.so >> $O/c5.log 2>&1 || exit 1
done
timeout -k 10 300 python tools/ablate.py $L/lib_base.so $L/lib_a2.so $L/lib_a3.so >> $O/c4.log 2>&1 || exit 2
cat $O/c5.log $O/c4.log
