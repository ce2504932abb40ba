#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03
HMGPU_LIB=hypermerge_amd/_lib/ablate/lib_stamps.so timeout -k 10 300 python tools/lstamps.py C3 10000 > gpurun_out/r03/lstamps_c3.log 2>&1 || { tail gpurun_out/r03/lstamps_c3.log; exit 2; }
grep -v amdgpu.ids gpurun_out/r03/lstamps_c3.log
