#!/bin/bash
# A/B of the ablate variants on C2 and C5 (kernel lines only)
set -o pipefail
mkdir -p gpurun_out/ab
LIBS=$(ls hypermerge_amd/_lib/ablate/lib_*.so | grep -v stamps)
ABL_CONFIG=C2 ABL_DOCS=100000 timeout -k 10 300 python tools/ablate.py $LIBS > gpurun_out/ab/c2.log 2>&1 || exit 4
echo "C2"; cat gpurun_out/ab/c2.log
ABL_CONFIG=C5 ABL_DOCS=100000 timeout -k 10 300 python tools/ablate.py $LIBS > gpurun_out/ab/c5.log 2>&1 || exit 5
echo "C5"; cat gpurun_out/ab/c5.log
