#!/bin/bash
# A/B round: parity tests on the default build, then every ablate variant on C4, C4 actor-major, C2, C5
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_store_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ab/tests.log; exit 1; }
tail -1 gpurun_out/ab/tests.log
LIBS=$(ls hypermerge_amd/_lib/ablate/lib_*.so | grep -v stamps)
for rep in 1 2; do
ABL_CONFIG=C4 timeout -k 10 600 python tools/ablate.py $LIBS > gpurun_out/ab/c4_$rep.log 2>&1 || exit 2
echo "C4 rep $rep"; cat gpurun_out/ab/c4_$rep.log
done
ABL_CONFIG=C4 ABL_ARGS="--arrival 1" timeout -k 10 600 python tools/ablate.py $LIBS > gpurun_out/ab/c4am.log 2>&1 || exit 3
echo "C4am"; cat gpurun_out/ab/c4am.log
ABL_CONFIG=C2 ABL_DOCS=100000 timeout -k 10 600 python tools/ablate.py $LIBS > gpurun_out/ab/c2.log 2>&1 || exit 4
echo "C2"; cat gpurun_out/ab/c2.log
ABL_CONFIG=C5 ABL_DOCS=100000 timeout -k 10 600 python tools/ablate.py $LIBS > gpurun_out/ab/c5.log 2>&1 || exit 5
echo "C5"; cat gpurun_out/ab/c5.log
