#!/bin/bash
# round 4: resident-store tests + incremental round phases (inc vs re-merge, host and device entry points)
set -o pipefail
OUT=gpurun_out/r04/${1:-store}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_store_gpu.py tests/test_general_resident.py tests/test_wide_gpu.py tests/test_docset_gpu.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 240 python tools/inc_profile.py --incremental 1 --device 1 > $OUT/inc_dev.log 2>&1 || { tail -20 $OUT/inc_dev.log; exit 2; }
timeout -k 10 240 python tools/inc_profile.py --incremental 0 --device 1 > $OUT/rem_dev.log 2>&1 || { tail -20 $OUT/rem_dev.log; exit 3; }
timeout -k 10 240 python tools/inc_profile.py --incremental 1 > $OUT/inc.log 2>&1 || { tail -20 $OUT/inc.log; exit 4; }
grep -v amdgpu.ids $OUT/inc_dev.log | tail -45
grep -v amdgpu.ids $OUT/rem_dev.log | tail -45
grep -v amdgpu.ids $OUT/inc.log | grep round
