#!/bin/bash
# CPU profile of the Node DocBackend legs (node --cpu-prof) on a C2 sample: where the
# per-document time of the JS restatement and of the GPU drop-in goes.
#   tools/node_profile.sh OUT NDOCS MODES
set -o pipefail
OUT=${1:-gpurun_out/node_prof}
N=${2:-20000}
MODES=${3:-gpu_async}
mkdir -p $OUT
python3 -c "
import json, sys
sys.path.insert(0, '.')
from hypermerge_amd import synth
from hypermerge_amd.columnar import decode_doc
b = synth.generate(synth.config('C2', n_docs=$N), threads=16)
docs = [decode_doc(b, i) for i in range(b.n_docs)]
json.dump({'docs': [[d[k:k + 16] for k in range(0, len(d), 16)] for d in docs]}, open('/tmp/hm_c2.json', 'w'))
" || exit 1
for m in ${MODES//,/ }; do
  timeout -k 10 300 node --cpu-prof --cpu-prof-dir $OUT/prof_$m tools/bench_node.js /tmp/hm_c2.json $m > $OUT/result_$m.json 2> $OUT/err_$m.log || exit 1
  python3 tools/cpuprofile_top.py $OUT/prof_$m/*.cpuprofile 40 > $OUT/top_$m.txt || exit 1
  rm -f $OUT/prof_$m/*.cpuprofile
done
rm -f /tmp/hm_c2.json
