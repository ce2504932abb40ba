#!/bin/bash
# A/B of the Node drop-in on one box: ab_old/ (previous JS + addon) vs the tree's, C2 20k async legs
set -o pipefail
O=gpurun_out/r03/node_ab
mkdir -p $O
python3 -c "
import json, sys
sys.path.insert(0, '.')
from hypermerge_amd import synth
from hypermerge_amd.columnar import decode_doc
b = synth.generate(synth.config('C2', n_docs=20000), threads=16)
docs = [decode_doc(b, i) for i in range(b.n_docs)]
json.dump({'docs': [[d[k:k + 16] for k in range(0, len(d), 16)] for d in docs]}, open('/tmp/hm_c2.json', 'w'))
" || exit 1
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export HM_GPU_JS=$PWD/ab_old/js/GpuDocBackend.js; else unset HM_GPU_JS; fi
    timeout -k 10 300 node --max-old-space-size=16384 tools/bench_node.js /tmp/hm_c2.json cpu,gpu_async > $O/$v$r.json 2> $O/$v$r.err || exit 1
    python3 -c "
import json; d=json.load(open('$O/$v$r.json'))
print('$v$r', ' '.join('%s %.3e' % (k, v['changes_per_s']) for k, v in d.items()), d['gpu_async'].get('state_digest'))
"
  done
done
rm -f /tmp/hm_c2.json
