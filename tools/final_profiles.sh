#!/bin/bash
# Round-end measurement at HEAD: the default bench line (all legs), rocprofv3 kernel stats + PMC of the
# C4, C3 and C5 steps.  Outputs under gpurun_out/<tag> (argument 1).
set -o pipefail
O=gpurun_out/${1:-final}
mkdir -p $O
if [ "$2" != "nobench" ]; then
timeout -k 10 900 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench_line.json
cp gpurun_out/bench_detail.json $O/bench_detail.json
fi
bash tools/profile.sh ${1:-final}_c4 > $O/profile_c4.log 2>&1 || { tail $O/profile_c4.log; exit 2; }
python tools/pmc_summary.py gpurun_out/${1:-final}_c4 > $O/c4_pmc_summary.json || exit 3
find gpurun_out/${1:-final}_c4/trace -name "*kernel_stats.csv" -exec cp {} $O/c4_kernel_stats.csv \;
bash tools/profile.sh ${1:-final}_c3 --config C3 --docs 10000 > $O/profile_c3.log 2>&1 || { tail $O/profile_c3.log; exit 4; }
python tools/pmc_summary.py gpurun_out/${1:-final}_c3 merge_large_kernel > $O/c3_pmc_summary.json || exit 5
find gpurun_out/${1:-final}_c3/trace -name "*kernel_stats.csv" -exec cp {} $O/c3_kernel_stats.csv \;
bash tools/profile.sh ${1:-final}_c5 --config C5 --docs 100000 > $O/profile_c5.log 2>&1 || { tail $O/profile_c5.log; exit 6; }
python tools/pmc_summary.py gpurun_out/${1:-final}_c5 > $O/c5_pmc_summary.json || exit 7
find gpurun_out/${1:-final}_c5/trace -name "*kernel_stats.csv" -exec cp {} $O/c5_kernel_stats.csv \;
python3 -c "
import json
import os
if os.path.exists('$O/bench_line.json'):
    d = json.load(open('$O/bench_line.json'))
    print('value %.4e ms %.3f frac %.4f' % (d['value'], d['ms_per_step'], d['roofline']['frac']))
for f in ('c4', 'c3', 'c5'):
    s = json.load(open('$O/%s_pmc_summary.json' % f))
    print(f, {k: round(v, 4) if isinstance(v, float) else v for k, v in s.items() if k in ('avg_ns', 'hbm_traffic_bytes', 'SQ_WAIT_ANY', 'SQ_WAVE_CYCLES', 'SQ_LDS_BANK_CONFLICT', 'SQ_INSTS_LDS')})
"
