#!/bin/bash
# Kernel-only bench lines for several configs (no CPU / PMC / side legs): tools/quick_cfg.sh OUT "C5:100000 C4:1000000 ..."
set -o pipefail
OUT=${1:-gpurun_out/quick}
mkdir -p $OUT
for spec in $2; do
  cfg=${spec%%:*}; n=${spec#*:}
  timeout -k 10 300 python bench.py --config $cfg --docs $n --steps 10 --warmup 2 --no-cpu --no-traffic --no-e2e --no-incremental --no-node --no-orders --check-docs 2000 > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/bench_$cfg.json').read().strip().splitlines()[-1]); print('$cfg', '%.4e' % d['value'], 'ms %.3f' % d['ms_per_step'], 'frac %.4f' % d['roofline']['frac'], 'parity', d['parity_sample_ok'], [(k['kernel'][6:11], round(k['ms'],3), k['docs']) for k in d['roofline']['kernels']])"
done
