#!/bin/bash
# Round-3 check after the block-decoder rework: GPU parity tests, then the default bench line
# (its from_blocks leg times the decoder on the box's host cores).
set -o pipefail
O=gpurun_out/r03/${FINAL_TAG:-dec}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
echo smoke ok
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 2; }
tail -1 $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.3e frac %.3f' % (d['value'], d['roofline']['frac'])); print('from_blocks', d.get('from_blocks'))"
