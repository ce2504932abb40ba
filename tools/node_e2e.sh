#!/bin/bash
# Node DocBackend end-to-end on a C2 sample (bench.py's node_docbackend leg, standalone).
set -o pipefail
OUT=${1:-gpurun_out/node_e2e}
N=${2:-2000}
mkdir -p $OUT
python3 -c "
import json, sys
sys.path.insert(0, '.')
from hypermerge_amd import synth
from hypermerge_amd.columnar import decode_doc
b = synth.generate(synth.config('C2', n_docs=$N))
docs = [decode_doc(b, i) for i in range(b.n_docs)]
json.dump({'docs': [[d[k:k + 16] for k in range(0, len(d), 16)] for d in docs]}, open('$OUT/c2.json', 'w'))
" && timeout -k 10 300 node tools/bench_node.js $OUT/c2.json cpu,gpu,gpu_async > $OUT/result.json
