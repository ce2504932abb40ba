#!/bin/bash
# round 4: per-phase cycle shares (HM_STAMPS build, shares only) of the small kernel on C4 / C5 and
# of the general kernel on C3
set -o pipefail
O=gpurun_out/r04/${1:-stamps}
mkdir -p $O
export HMGPU_LIB=hypermerge_amd/_lib/ablate/lib_stamps.so
timeout -k 10 200 python tools/stamps.py C4 1000000 > $O/stamps_c4.log 2>&1 || exit 2
timeout -k 10 200 python tools/stamps.py C5 100000 > $O/stamps_c5.log 2>&1 || exit 3
timeout -k 10 300 python tools/lstamps.py C3 10000 > $O/lstamps_c3.log 2>&1 || exit 4
grep -v amdgpu.ids $O/stamps_c4.log $O/stamps_c5.log $O/lstamps_c3.log
