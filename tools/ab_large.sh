#!/bin/bash
# general-kernel A/B: its parity tests on the default build, then the variants on C3 (x2) and C1
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_general_resident.py tests/test_wide_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ab/tests.log; exit 1; }
tail -1 gpurun_out/ab/tests.log
LIBS=$(ls hypermerge_amd/_lib/ablate/lib_*.so | grep -v stamps)
for rep in 1 2; do
ABL_CONFIG=C3 ABL_DOCS=10000 timeout -k 10 300 python tools/ablate.py $LIBS > gpurun_out/ab/c3_$rep.log 2>&1 || exit 5
echo "C3 rep $rep"; cat gpurun_out/ab/c3_$rep.log
done
ABL_CONFIG=C1 ABL_DOCS=1 ABL_ARGS="--arrival 1" timeout -k 10 300 python tools/ablate.py $LIBS > gpurun_out/ab/c1.log 2>&1 || exit 6
echo "C1am"; cat gpurun_out/ab/c1.log
