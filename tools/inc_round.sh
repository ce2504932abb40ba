#!/bin/bash
# Incremental rounds (new rows already in HBM) under rocprofv3: optional store/docset GPU tests,
# the per-phase log, kernel stats, PMC FETCH_SIZE / WRITE_SIZE.
#   tools/inc_round.sh <tag> [tests|notests|nopmc] [inc_profile.py args...]
set -o pipefail
OUT=gpurun_out/${1:-incprof}
MODE=${2:-tests}
shift 2
R=$PWD
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$MODE" = "tests" ]; then
  timeout -k 10 500 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_store_gpu.py tests/test_docset_gpu.py tests/test_general_resident.py > $OUT/tests.log 2>&1 || { grep -E "FAILED|Error|error" $OUT/tests.log | head -30; tail -40 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
timeout -k 10 240 python tools/inc_profile.py --incremental 1 --device 1 "$@" > $OUT/inc_dev.log 2>&1 || { tail -20 $OUT/inc_dev.log; exit 2; }
grep -v amdgpu.ids $OUT/inc_dev.log | tail -36
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/trace -o run -- python3 $R/tools/inc_profile.py --incremental 1 --device 1 "$@" > $R/$OUT/trace.log 2>&1 || exit 3
cd $R
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); head -16 $f | cut -c1-200
[ "$MODE" = "nopmc" ] && exit 0
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $R/$OUT/pmc_$C -o run -- python3 $R/tools/inc_profile.py --incremental 1 --device 1 "$@" > $R/$OUT/pmc_$C.log 2>&1 || exit 4
done
cd $R
for C in FETCH_SIZE WRITE_SIZE; do
  python3 - "$OUT/pmc_$C" "$C" <<'PY'
import csv, glob, sys, collections
d, c = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(list)
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if row.get("Counter_Name") == c:
            acc[row["Kernel_Name"][:60]].append((float(row["Counter_Value"]), int(row["Grid_Size"])))
for k, v in sorted(acc.items(), key=lambda x: -sum(a for a, _ in x[1])):
    print(c, k, "calls", len(v), "KiB/grid:", [(round(a), g) for a, g in v][:6])
PY
done
