#!/bin/bash
set -o pipefail
O=gpurun_out/r04/${1:-stamps5}
mkdir -p $O
export HMGPU_LIB=hypermerge_amd/_lib/ablate/lib_stamps.so
timeout -k 10 200 python tools/stamps.py C5 100000 > $O/stamps_c5.log 2>&1 || exit 3
grep -v amdgpu.ids $O/stamps_c5.log
