#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03
HMGPU_LIB=hypermerge_amd/_lib/ablate/lib_stamps.so timeout -k 10 200 python tools/stamps.py C5 100000 > gpurun_out/r03/stamps_c5.log 2>&1 || exit 2
grep -v amdgpu.ids gpurun_out/r03/stamps_c5.log
