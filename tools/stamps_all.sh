#!/bin/bash
# Phase shares (diagnostic HM_STAMPS=1 build, tools/build_variants.sh stamps:-DHM_STAMPS=1) of the
# C4 (generation and actor-major), C5 and C3 kernels.  Outputs under gpurun_out/<tag>.
set -o pipefail
O=gpurun_out/${1:-stamps}
mkdir -p $O
export HMGPU_LIB=hypermerge_amd/_lib/ablate/lib_stamps.so
timeout -k 10 180 python -u tools/stamps.py C4 1000000 > $O/c4.txt 2>&1 && cat $O/c4.txt &&
timeout -k 10 180 python -u tools/stamps.py C4 1000000 1 > $O/c4_am.txt 2>&1 && cat $O/c4_am.txt &&
timeout -k 10 180 python -u tools/stamps.py C5 100000 > $O/c5.txt 2>&1 && cat $O/c5.txt &&
timeout -k 10 180 python -u tools/lstamps.py C3 10000 > $O/c3.txt 2>&1 && cat $O/c3.txt
