#!/bin/bash
set -o pipefail
bash tools/ab_large.sh || exit 1
timeout -k 10 400 python -u -m pytest tests/test_store_gpu.py tests/test_docset_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/store_tests.log 2>&1 || { echo "store tests failed"; tail -30 gpurun_out/ab/store_tests.log; exit 2; }
tail -1 gpurun_out/ab/store_tests.log
bash tools/store_round.sh > gpurun_out/ab/store_round.txt 2>&1 || { tail -20 gpurun_out/ab/store_round.txt; exit 3; }
grep -E "round|plan|incremental |remerge " gpurun_out/ab/store_round.txt | head -24
grep -E "plan_kernel|doc_rows|inc_apply" gpurun_out/r03/store/trace/run_kernel_stats.csv
