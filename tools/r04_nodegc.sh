#!/bin/bash
# round 4: V8 GC trace of the Node gpu_async leg (C2 20k): scavenges vs mark-compacts
set -o pipefail
O=gpurun_out/r04/${1:-nodegc}
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
timeout -k 10 120 node --max-old-space-size=16384 --max-semi-space-size=64 --trace-gc tools/bench_node.js /tmp/hm_c2.json gpu_async > $O/gc_gpu.log 2>&1 || exit 3
timeout -k 10 120 node --max-old-space-size=16384 --max-semi-space-size=64 --trace-gc tools/bench_node.js /tmp/hm_c2.json cpu > $O/gc_cpu.log 2>&1 || exit 4
for f in gc_gpu gc_cpu; do
  echo $f; grep -c Scavenge $O/$f.log; grep -c "Mark-Compact\|Mark-sweep" $O/$f.log; tail -1 $O/$f.log | cut -c1-300
done
rm -f /tmp/hm_c2.json
