#!/bin/bash
# SQ / TA counters of the incremental kernels (tools/inc_profile.py rounds), one rocprofv3 pass
# per counter group.  tools/inc_pmc.sh <tag> [inc_profile.py args...]; HM_INC_LANE picks the pass.
set -o pipefail
OUT=gpurun_out/${1:-incpmc}
shift
R=$PWD
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for CS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
          "SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM TA_BUSY_avr TA_BUSY_max"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $CS --output-format csv -d $R/$OUT/p$i -o run -- python3 $R/tools/inc_profile.py --incremental 1 --device 1 "$@" > $R/$OUT/p$i.log 2>&1 || { tail -5 $R/$OUT/p$i.log; exit $i; }
done
cd $R
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + "/p*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        if "inc_" not in k or int(row["Grid_Size"]) < 500000:
            continue
        acc[k[:40]][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, m in acc.items():
    v = {c: sum(x) / len(x) for c, x in m.items()}
    print(k, {c: round(x) for c, x in v.items()})
    if "SQ_WAVE_CYCLES" in v and "SQ_WAIT_ANY" in v:
        print("   wait_any/wave_cycles %.3f  active_inst/wave_cycles %.3f" % (v["SQ_WAIT_ANY"] / v["SQ_WAVE_CYCLES"], v.get("SQ_ACTIVE_INST_ANY", 0) / v["SQ_WAVE_CYCLES"]))
PY
