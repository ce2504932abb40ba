#!/bin/bash
# round 4: incremental rounds (device-resident rows) under rocprofv3: kernel stats + PMC traffic
set -o pipefail
OUT=gpurun_out/r04/${1:-incprof}
R=$PWD
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${2:-tests}" = "tests" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_store_gpu.py tests/test_docset_gpu.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
timeout -k 10 240 python tools/inc_profile.py --incremental 1 --device 1 > $OUT/inc_dev.log 2>&1 || { tail -20 $OUT/inc_dev.log; exit 2; }
grep -v amdgpu.ids $OUT/inc_dev.log | tail -36
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/trace -o run -- python3 $R/tools/inc_profile.py --incremental 1 --device 1 > $R/$OUT/trace.log 2>&1 || exit 3
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $R/$OUT/pmc_$C -o run -- python3 $R/tools/inc_profile.py --incremental 1 --device 1 > $R/$OUT/pmc_$C.log 2>&1 || exit 4
done
cd $R
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); head -14 $f
for C in FETCH_SIZE WRITE_SIZE; do
  python3 - "$OUT/pmc_$C" "$C" <<'PY'
import csv, glob, sys, collections
d, c = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(list)
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if row.get("Counter_Name") == c:
            acc[row["Kernel_Name"][:60]].append(float(row["Counter_Value"]))
for k, v in sorted(acc.items(), key=lambda x: -sum(x[1])):
    print(c, k, "calls", len(v), "avg KiB", sum(v) / len(v))
PY
done
