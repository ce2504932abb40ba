#!/bin/bash
# round 4: A/B of the Node drop-in: HEAD's GpuDocBackend (js/GpuDocBackend_base.js) vs the working
# copy, gpu_async legs alternating in separate processes on one box, cpu once
set -o pipefail
O=gpurun_out/r04/${1:-nodeab}
mkdir -p $O
python3 -c "
import json, sys
sys.path.insert(0, '.')
from hypermerge_amd import synth
from hypermerge_amd.columnar import decode_doc
b = synth.generate(synth.config('C2', n_docs=20000), threads=16)
docs = [decode_doc(b, i) for i in range(b.n_docs)]
json.dump({'docs': [[d[k:k + 16] for k in range(0, len(d), 16)] for d in docs]}, open('/tmp/hm_c2.json', 'w'))
" || exit 2
N="node --max-old-space-size=16384 --max-semi-space-size=64 tools/bench_node.js /tmp/hm_c2.json"
timeout -k 10 120 $N cpu > $O/cpu.json 2>/dev/null || exit 3
for i in 1 2 3; do
  HM_GPU_JS=$PWD/hypermerge_amd/js/GpuDocBackend_base.js timeout -k 10 120 $N gpu_async > $O/base$i.json 2>/dev/null || exit 4
  timeout -k 10 120 $N gpu_async > $O/new$i.json 2>/dev/null || exit 5
done
python3 -c "
import json
r = lambda f: json.load(open('$O/' + f))
print('cpu', round(r('cpu.json')['cpu']['changes_per_s']))
for i in (1, 2, 3):
    b, n = r('base%d.json' % i)['gpu_async'], r('new%d.json' % i)['gpu_async']
    print(i, 'base', round(b['changes_per_s']), 'new', round(n['changes_per_s']), b['state_digest'] == n['state_digest'])
"
rm -f /tmp/hm_c2.json
