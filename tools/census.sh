#!/bin/bash
# Dynamic instruction census of merge_small_kernel by phase: for each library (an HM_ABLATE
# early-exit build from tools/build_variants.sh, or the full build), one PMC pass over
# tools/census.py; prints VALU / SALU / LDS instructions and wave cycles per document.
#   tools/census.sh <tag> <config> <docs> [arrival] -- lib1.so lib2.so ...
set -o pipefail
O=$PWD/gpurun_out/${1:-census}; CFG=$2; N=$3; shift 3
ARR=""
if [ "$1" != "--" ]; then ARR=$1; shift; fi
shift
R=$PWD
mkdir -p $O
export TMPDIR=/tmp
for so in "$@"; do
  b=$(basename $so .so)
  (cd /tmp && HMGPU_LIB=$R/$so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d $O/$b -o run -- python3 $R/tools/census.py $CFG $N $ARR > $O/$b.log 2>&1) || { tail -5 $O/$b.log; exit 1; }
  python3 - $O/$b $b $N <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "merge_small_kernel" in row.get("Kernel_Name", ""):
            acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
n = float(sys.argv[3])
v = {k: sum(x) / len(x) for k, x in acc.items()}
print("%-12s VALU/doc %7.1f  SALU/doc %7.1f  LDS/doc %6.1f  wave_cycles/doc %9.1f  wait %.3f" % (
    sys.argv[2], v.get("SQ_INSTS_VALU", 0) / n, v.get("SQ_INSTS_SALU", 0) / n, v.get("SQ_INSTS_LDS", 0) / n,
    v.get("SQ_WAVE_CYCLES", 0) / n, v.get("SQ_WAIT_ANY", 0) / max(1, v.get("SQ_WAVE_CYCLES", 1))), flush=True)
PY
done
