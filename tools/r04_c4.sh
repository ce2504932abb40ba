#!/bin/bash
# round 4: small-kernel change check — parity suite, then the C4 kernel's trace + LDS/SQ counters
set -o pipefail
TAG=${1:-c4}
O=gpurun_out/r04/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
R=$PWD
ARGS="--steps 3 --warmup 1 --no-cpu --no-traffic --no-e2e --no-orders --no-incremental --no-node --check-docs 0 ${2:-}"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o run -- python3 $R/bench.py $ARGS > $R/$O/trace.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $R/$O/pmc1 -o run -- python3 $R/bench.py $ARGS > $R/$O/pmc1.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d $R/$O/pmc2 -o run -- python3 $R/bench.py $ARGS > $R/$O/pmc2.log 2>&1 || exit 4
cd $R
python tools/pmc_summary.py $O > $O/pmc_summary.json || exit 5
grep '^{' $O/trace.log | tail -1 > $O/bench_line.json
python3 -c "
import json
s = json.load(open('$O/pmc_summary.json'))
d = json.load(open('$O/bench_line.json'))
print('value %.4e frac %.4f' % (d['value'], d['roofline']['frac']))
print({k: s.get(k) for k in ('avg_ns', 'SQ_WAIT_ANY', 'SQ_WAVE_CYCLES', 'SQ_LDS_BANK_CONFLICT', 'SQ_INSTS_LDS')})
print('wait/cycles %.3f conflicts/lds %.3f' % (s['SQ_WAIT_ANY'] / s['SQ_WAVE_CYCLES'], s['SQ_LDS_BANK_CONFLICT'] / s['SQ_INSTS_LDS']))
"
