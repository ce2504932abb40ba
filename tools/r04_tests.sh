#!/bin/bash
# round 4: GPU tests of the resident store, docset and Node drop-in
set -o pipefail
OUT=gpurun_out/r04/${1:-tests}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread ${2:-tests/test_store_gpu.py tests/test_docset_gpu.py tests/test_node_gpu.py} > $OUT/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" $OUT/tests.log | tail -60
tail -3 $OUT/tests.log
exit $rc
