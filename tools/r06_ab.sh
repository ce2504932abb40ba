#!/bin/bash
# dev A/B of small-kernel variants on C4, C4 actor-major and C5 (tools/ablate.py, alternating reps)
OUT=gpurun_out/${1:-ab}; shift
mkdir -p $OUT
L=""; for v in "$@"; do L="$L hypermerge_amd/_lib/ablate/lib_$v.so"; done
ABL_REPS=2 timeout -k 10 280 python tools/ablate.py $L > $OUT/c4.txt 2>&1 || exit 1
ABL_REPS=2 ABL_ARGS="--arrival 1" timeout -k 10 280 python tools/ablate.py $L > $OUT/c4am.txt 2>&1 || exit 1
ABL_REPS=2 ABL_CONFIG=C5 ABL_DOCS=100000 timeout -k 10 200 python tools/ablate.py $L > $OUT/c5.txt 2>&1 || exit 1
cat $OUT/c4.txt $OUT/c4am.txt $OUT/c5.txt
