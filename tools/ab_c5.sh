#!/bin/bash
# C5-focused A/B: list parity tests on the default build, then the variants on C5 (x2) and C4
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_general_resident.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ab/tests.log; exit 1; }
tail -1 gpurun_out/ab/tests.log
LIBS=$(ls hypermerge_amd/_lib/ablate/lib_*.so | grep -v stamps)
for rep in 1 2; do
ABL_CONFIG=C5 ABL_DOCS=100000 timeout -k 10 300 python tools/ablate.py $LIBS > gpurun_out/ab/c5_$rep.log 2>&1 || exit 5
echo "C5 rep $rep"; cat gpurun_out/ab/c5_$rep.log
done
ABL_CONFIG=C4 timeout -k 10 300 python tools/ablate.py $LIBS > gpurun_out/ab/c4.log 2>&1 || exit 6
echo "C4"; cat gpurun_out/ab/c4.log
