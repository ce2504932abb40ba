#!/bin/bash
# round 4: Node drop-in checks — the Node GPU tests, then the C2 legs (cpu once, gpu_async x3) under
# two V8 young-generation sizes
set -o pipefail
O=gpurun_out/r04/${1:-node}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_node_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
python3 -c "
import json, sys
sys.path.insert(0, '.')
from hypermerge_amd import synth
from hypermerge_amd.columnar import decode_doc
b = synth.generate(synth.config('C2', n_docs=20000), threads=16)
docs = [decode_doc(b, i) for i in range(b.n_docs)]
json.dump({'docs': [[d[k:k + 16] for k in range(0, len(d), 16)] for d in docs]}, open('/tmp/hm_c2.json', 'w'))
" || exit 2
for semi in 64 128; do
  timeout -k 10 300 node --max-old-space-size=16384 --max-semi-space-size=$semi tools/bench_node.js /tmp/hm_c2.json cpu,gpu_async,gpu_async,gpu_async > $O/legs_$semi.json 2> $O/legs_$semi.err || exit 3
  python3 -c "
import json; d = json.load(open('$O/legs_$semi.json'))
print('semi $semi', {k: round(v['changes_per_s']) for k, v in d.items()})
"
done
rm -f /tmp/hm_c2.json
