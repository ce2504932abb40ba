#!/bin/bash
# round 4: the default bench line (as the driver runs it) + GPU tests log
set -o pipefail
OUT=gpurun_out/r04/${1:-bench}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log > $OUT/bench_line.json
python -c "
import json
d=json.load(open('$OUT/bench_line.json'))
print('value', d['value'], 'frac', d['roofline']['frac'], 'kernel_ms', d['roofline']['kernel_ms'])
ri=d.get('resident_incremental') or {}
print('inc', {k: ri.get(k) for k in ('value','remerge_value','speedup_vs_remerge','same_as_remerge','all_incremental','pcie_value','us_per_round')})
for r in ri.get('rounds', []): print(r['docs'], r['incremental']['ms'], r['remerge']['ms'], r['pcie_incremental']['ms'])
nd=d.get('node_docbackend') or {}
rt=d.get('resident_incremental_text') or {}
print('text', {k: rt.get(k) for k in ('value','remerge_value','speedup_vs_remerge','same_as_remerge','all_incremental','incremental_share','oracle_docs_equal','us_per_round')})
for r in rt.get('rounds', []): print(r['docs'], r['incremental']['ms'], r['remerge']['ms'])
r5=d.get('resident_incremental_c5') or {}
print('c5', {k: r5.get(k) for k in ('value','remerge_value','speedup_vs_remerge','same_as_remerge','incremental_share','bail_share','oracle_docs_equal')})
print('node', {k: nd.get(k) for k in ('gpu_async_vs_js','gpu_async_vs_js_blocks','same_state','same_clocks')}, {c: {k: (nd.get(c) or {}).get(k) for k in ('gpu_async_vs_js','same_state','same_clocks','error')} for c in ('C3','C5')})
"
