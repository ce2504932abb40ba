#!/bin/bash
# The Node DocBackend legs on a C2 sample (tools/bench_node.js), then a CPU profile
# (node --cpu-prof) of the chosen legs: where the per-document time goes.
#   tools/node_profile.sh OUT NDOCS BENCH_LEGS PROFILE_LEGS
set -o pipefail
OUT=${1:-gpurun_out/node_prof}
N=${2:-20000}
LEGS=${3:-cpu,cpu_blocks,gpu,gpu_async,gpu_objects}
PLEGS=${4:-gpu_async}
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
HM_DOCSET_PROFILE=1 timeout -k 10 600 node --max-old-space-size=16384 --max-semi-space-size=64 tools/bench_node.js /tmp/hm_c2.json $LEGS > $OUT/bench.json 2> $OUT/bench_err.log || exit 1
for m in ${PLEGS//,/ }; do
  sleep 3
  HM_NODE_PROF=/tmp/hm_$m.cpuprofile timeout -k 10 300 node --max-old-space-size=16384 --max-semi-space-size=64 tools/bench_node.js /tmp/hm_c2.json $m > $OUT/result_$m.json 2> $OUT/err_$m.log || exit 1
  python3 tools/cpuprofile_top.py /tmp/hm_$m.cpuprofile 40 > $OUT/top_$m.txt || exit 1
  rm -f /tmp/hm_$m.cpuprofile
done
rm -f /tmp/hm_c2.json
