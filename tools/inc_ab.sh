#!/bin/bash
# A/B of library builds on the resident incremental rounds (dev): tools/inc_ab.sh <out> lib1.so lib2.so ...
# each library runs tools/inc_profile.py (1M C4 documents, rows in HBM) twice, alternating.
OUT=gpurun_out/${1:-incab}; shift
mkdir -p $OUT
for rep in 1 2; do
  for so in "$@"; do
    n=$(basename $so .so)
    HMGPU_LIB=$(realpath $so) timeout -k 10 200 python tools/inc_profile.py --device 1 > $OUT/${n}_$rep.log 2>&1 || { tail -5 $OUT/${n}_$rep.log; exit 1; }
    echo "$n rep $rep: $(grep -E '^\[hm_store\] incremental' $OUT/${n}_$rep.log | awk '{print $3}' | tr '\n' ' ')"
  done
done
