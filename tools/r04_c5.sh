#!/bin/bash
# round 4: small-kernel list launches — parity suites touching lists, then the C5 kernel's trace + counters
set -o pipefail
TAG=${1:-c5}
O=gpurun_out/r04/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_store_gpu.py > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
R=$PWD
ARGS="--steps 3 --warmup 1 --no-cpu --no-traffic --no-e2e --no-orders --no-incremental --no-node --check-docs 0 --config C5 --docs 100000"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o run -- python3 $R/bench.py $ARGS > $R/$O/trace.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $R/$O/pmc1 -o run -- python3 $R/bench.py $ARGS > $R/$O/pmc1.log 2>&1 || exit 3
cd $R
python tools/pmc_summary.py $O > $O/pmc_summary.json || exit 5
python3 -c "
import json
s = json.load(open('$O/pmc_summary.json'))
print({k: s.get(k) for k in ('avg_ns', 'calls', 'SQ_WAVES', 'SQ_WAIT_ANY', 'SQ_WAVE_CYCLES')})
print('wait/cycles %.3f' % (s['SQ_WAIT_ANY'] / s['SQ_WAVE_CYCLES']))
"
grep -h "merge_small\|merge_large" $O/trace/*kernel_stats.csv | cut -c1-160
