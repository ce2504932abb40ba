#!/bin/bash
# Node C2 20k legs only (no tests)
set -o pipefail
bash tools/node_profile.sh gpurun_out/r03/node 20000 ${1:-cpu,gpu_async,gpu_async_net} gpu_async || exit 2
python3 -c "
import json; d=json.load(open('gpurun_out/r03/node/bench.json'))
for k,v in d.items(): print(k, '%.3e'%v['changes_per_s'], v['diffs'])
"
