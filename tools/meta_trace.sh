#!/bin/bash
# inc_meta_kernel / doc_rows_kernel durations per call on the C4 (1M) and C5 (100k) resident
# rounds of tools/inc_profile.py (rocprofv3 kernel trace).  tools/meta_trace.sh <out>
set -o pipefail
OUT=gpurun_out/${1:-metatrace}
R=$PWD
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/c4 -o run -- python3 $R/tools/inc_profile.py --device 1 > $R/$OUT/c4.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/c5 -o run -- python3 $R/tools/inc_profile.py --config C5 --docs 100000 --device 1 --incremental 1 > $R/$OUT/c5.log 2>&1 || exit 2
cd $R
for c in c4 c5; do
  echo "== $c"
  python3 - $(find $OUT/$c -name "*kernel_trace.csv" | head -1) <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Kernel_Name']
    if 'inc_meta' in n or 'doc_rows' in n or 'inc_group_kernel<8' in n:
        print('%-34s %9.1f us' % (n[:34], (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3))
PY
done
