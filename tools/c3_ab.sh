#!/bin/bash
# A/B of library builds on the resident C3 rounds: the wave pass's kernel time per round
# (rocprofv3 kernel trace).  tools/c3_ab.sh <out> lib1.so lib2.so ...
set -o pipefail
OUT=gpurun_out/${1:-c3ab}; shift
R=$PWD
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for so in "$@"; do
    n=$(basename $so .so)
    cd /tmp
    HMGPU_LIB=$(realpath $R/$so) timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/${n}_$rep -o run -- python3 $R/tools/inc_profile.py --config C3 --docs 10000 --device 1 > $R/$OUT/${n}_$rep.log 2>&1 || exit 1
    cd $R
    echo "$n rep $rep: $(python3 - $(find $OUT/${n}_$rep -name '*kernel_trace.csv' | head -1) <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
print(' '.join('%.1f' % ((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3) for r in rows if 'inc_group_kernel<64, false' in r['Kernel_Name']))
PY
)"
  done
done
