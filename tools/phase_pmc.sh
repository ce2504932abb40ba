#!/bin/bash
# Per-phase instruction counts of merge_small_kernel from ablation builds (tools/build_variants.sh
# s008:-DHM_ABLATE=8 ...): one rocprofv3 PMC pass per library.  Usage: tools/phase_pmc.sh <tag> lib...
set -o pipefail
TAG=$1; shift
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for so in "$@"; do
  n=$(basename $so .so)
  HMGPU_LIB=$R/$so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_IFETCH --output-format csv -d $OUT/$n -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-traffic --no-e2e --no-orders --check-docs 0 > $OUT/$n.log 2>&1 || exit 1
  python3 $R/tools/pmc_summary.py $OUT/$n > $OUT/$n.json
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', ' '.join(f'{k}={v/1e6:.1f}' for k,v in sorted(d.items())))"
done
