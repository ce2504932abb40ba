#!/bin/bash
# Per-phase instruction counts: one PMC pass per ablation build (hypermerge_amd/_lib/ablate/lib_aNNN.so),
# merge_small_kernel only.  Differences between consecutive stop points = the phase's counts.
set -o pipefail
R=$PWD
mkdir -p gpurun_out/phase
export TMPDIR=/tmp
for so in ${@:-$R/hypermerge_amd/_lib/ablate/lib_a*.so}; do
  t=$(basename $so .so)
  ( cd /tmp && HMGPU_LIB=$so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD --output-format csv -d $R/gpurun_out/phase/$t -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/phase/$t.log 2>&1 ) || { echo "fail $t"; exit 1; }
  python3 - $R/gpurun_out/phase/$t <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "merge_small_kernel" in row["Kernel_Name"]:
            acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
print(sys.argv[1].split("/")[-1], " ".join(f"{k}={sum(v)/len(v)/1e6:.1f}" for k, v in sorted(acc.items())), "(per launch /1e6 ~ per doc)")
PY
done
