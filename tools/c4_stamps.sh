#!/bin/bash
# merge_small_kernel phase shares (HM_STAMPS build) on C4, generation order and actor-major
set -o pipefail
mkdir -p gpurun_out/r03
HMGPU_LIB=hypermerge_amd/_lib/ablate/lib_stamps.so timeout -k 10 200 python tools/stamps.py C4 1000000 > gpurun_out/r03/stamps_c4.log 2>&1 || exit 2
HMGPU_LIB=hypermerge_amd/_lib/ablate/lib_stamps.so timeout -k 10 200 python tools/stamps.py C4 1000000 1 > gpurun_out/r03/stamps_c4am.log 2>&1 || exit 3
HMGPU_LIB=hypermerge_amd/_lib/ablate/lib_stamps.so timeout -k 10 200 python tools/stamps.py C2 100000 > gpurun_out/r03/stamps_c2.log 2>&1 || exit 4
grep -v amdgpu.ids gpurun_out/r03/stamps_c4.log; grep -v amdgpu.ids gpurun_out/r03/stamps_c4am.log; grep -v amdgpu.ids gpurun_out/r03/stamps_c2.log
