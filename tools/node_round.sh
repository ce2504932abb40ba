#!/bin/bash
# Node drop-in: GPU tests of the Node host, then the C2 20k-document legs and a CPU profile
set -o pipefail
bash tools/t_quick.sh "node or docset" || exit 1
bash tools/node_profile.sh gpurun_out/r03/node 20000 ${1:-cpu,gpu,gpu_async,gpu_async_net} gpu_async || exit 2
python3 -c "
import json; d=json.load(open('gpurun_out/r03/node/bench.json'))
for k,v in d.items(): print(k, '%.3e'%v['changes_per_s'], v['diffs'], v.get('state_digest'), v.get('digest'))
"
head -12 gpurun_out/r03/node/top_gpu_async.txt
