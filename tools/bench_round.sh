#!/bin/bash
# The default bench line (every leg) under a time limit; $1 = output dir under gpurun_out/
set -o pipefail
O=gpurun_out/${1:-bench}
mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench_line.json
python3 -c "
import json
d = json.load(open('$O/bench_line.json'))
print('value %.4e ms %.3f frac %.4f traffic %s' % (d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic']))
for k in ('resident_incremental', 'resident_incremental_text', 'resident_incremental_c5'):
    r = d.get(k) or {}
    print(k, {x: r.get(x) for x in ('value', 'speedup_vs_remerge', 'incremental_share', 'us_per_round', 'same_as_remerge', 'oracle_docs_equal')}, (r.get('roofline') or {}).get('frac'), (r.get('roofline') or {}).get('traffic_vs_alg'))
n = d.get('node_docbackend') or {}
print('node', {k: n.get(k) for k in ('gpu_async_vs_js', 'gpu_async_vs_js_blocks', 'same_state')}, {k: (n.get(k) or {}).get('gpu_async_vs_js') for k in ('C3', 'C5')})
"
