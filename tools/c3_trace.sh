#!/bin/bash
# Kernel trace of the resident C3 rounds (tools/inc_profile.py --config C3, 10k text documents):
# every kernel's duration in launch order.  tools/c3_trace.sh <out>
set -o pipefail
OUT=gpurun_out/${1:-c3trace}
R=$PWD
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/t -o run -- python3 $R/tools/inc_profile.py --config C3 --docs 10000 --device 1 > $R/$OUT/c3.log 2>&1 || exit 1
cd $R
python3 - $(find $OUT/t -name "*kernel_trace.csv" | head -1) > $OUT/kernels.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
t0 = int(rows[0]['Start_Timestamp'])
for r in rows:
    print('%10.1f  %9.1f us  %s' % ((int(r['Start_Timestamp']) - t0) / 1e3, (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3, r['Kernel_Name'][:70]))
PY
grep -E "round|inc_states" $OUT/c3.log | cut -c1-200
tail -60 $OUT/kernels.txt
