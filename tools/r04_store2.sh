#!/bin/bash
# round 4: store GPU tests, the append census, then the default bench line
set -o pipefail
O=gpurun_out/r04/store2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_store_gpu.py tests/test_docset_gpu.py tests/test_node_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/r04_census.sh > $O/census.log 2>&1 || { tail -30 $O/census.log; exit 2; }
grep -h "append:" gpurun_out/r04/census/c5.log gpurun_out/r04/census/c4.log
timeout -k 10 700 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 3; }
grep '^{' $O/bench.log | tail -1 > $O/bench_line.json
python3 -c "
import json
d = json.load(open('$O/bench_line.json'))
print('value %.4e frac %.4f' % (d['value'], d['roofline']['frac']))
for k in ('resident_incremental', 'resident_incremental_text', 'resident_incremental_c5'):
    r = d[k]; print(k, '%.3e' % r['value'], 'remerge %.3e' % r['remerge_value'], 'x%.2f' % r['speedup_vs_remerge'], 'us/round %.0f' % r['us_per_round'], [round(x['incremental']['ms'], 3) for x in r['rounds']], [round(x['remerge']['ms'], 3) for x in r['rounds']])
"
