#!/bin/bash
# round 4: A/B of the ablate variants (kernel lines only) on C5 (and C2), twice each in alternation
set -o pipefail
O=gpurun_out/r04/${1:-ab}
mkdir -p $O
LIBS=$(ls hypermerge_amd/_lib/ablate/lib_*.so | grep -v stamps)
for cfg in ${2:-C5}; do
  ABL_CONFIG=$cfg ABL_DOCS=${3:-100000} timeout -k 10 500 python tools/ablate.py $LIBS $LIBS > $O/$cfg.log 2>&1 || exit 4
  echo $cfg; cat $O/$cfg.log
done
