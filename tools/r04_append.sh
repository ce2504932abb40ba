#!/bin/bash
# round 4: the store / docset GPU tests, then the C5 resident rounds' kernels (append_kernel<G>,
# plan launch width)
set -o pipefail
O=gpurun_out/r04/append
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_store_gpu.py tests/test_docset_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
bash tools/r04_c5ovh.sh
