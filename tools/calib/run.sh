#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration for scattered row accesses (tools/calib/fetch_calib.hip):
# one PMC pass per counter, then counter bytes / algorithmic bytes per kernel.
#   build (CPU): tools/calib/run.sh build     run (GPU box): tools/calib/run.sh <tag>
set -o pipefail
R="$(cd "$(dirname "$0")/../.." && pwd)"
BIN=$R/hypermerge_amd/_lib/fetch_calib
if [ "$1" = "build" ]; then
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -o $BIN $R/tools/calib/fetch_calib.hip
  exit $?
fi
O=$R/gpurun_out/${1:-calib}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 60 $BIN > $O/plain.log 2>&1 || { cat $O/plain.log; exit 1; }
cat $O/plain.log
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/$C -o run -- $BIN > $O/$C.log 2>&1 || { tail -5 $O/$C.log; exit 2; }
done
python3 - $O <<'PY'
import csv, glob, re, sys
from collections import defaultdict
O = sys.argv[1]
alg = {}
for l in open(O + "/plain.log"):
    m = re.match(r"(\S+)\s+algorithmic\s+(\d+) B", l)
    if m: alg[m.group(1)] = int(m.group(2))
val = defaultdict(dict)
for C in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(O + "/" + C + "/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            nm = "rd_stream_16B" if "rd_stream" in k else None
            m = re.search(r"(rd|wr)_lines<(\d+), (\d+)>", k)
            if m: nm = "%s_%sx%sB" % m.groups()
            if nm: val[nm][C] = val[nm].get(C, 0.0) + float(row["Counter_Value"]) * 1024
for nm, b in alg.items():
    key = "FETCH_SIZE" if nm.startswith("rd") else "WRITE_SIZE"
    x = val.get(nm, {}).get(key, 0.0)
    m = re.match(r"(rd|wr)_(\d+)x(\d+)B", nm)
    per_line = " per 128-B line touched %6.1f B" % (x / (b / (int(m.group(2)) * int(m.group(3))))) if m else ""
    print("%-16s alg %11d B  %s %13.0f B  counter/alg %.3f%s" % (nm, b, key, x, x / b, per_line))
PY
