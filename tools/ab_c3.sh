#!/bin/bash
# C3 (general kernel) A/B of the ablate variants
set -o pipefail
mkdir -p gpurun_out/ab
LIBS=$(ls hypermerge_amd/_lib/ablate/lib_*.so | grep -v stamps)
ABL_CONFIG=C3 ABL_DOCS=10000 timeout -k 10 400 python tools/ablate.py $LIBS > gpurun_out/ab/c3.log 2>&1 || { cat gpurun_out/ab/c3.log; exit 4; }
echo "C3"; cat gpurun_out/ab/c3.log
