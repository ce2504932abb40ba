#!/bin/bash
# A/B of the queued-history variants (tools/build_variants.sh libs): C4 actor-major, C5, C4 generation
set -o pipefail
O=gpurun_out/${1:-ab_hist}
shift
mkdir -p $O
ABL_ARGS="--arrival 1" timeout -k 10 300 python tools/ablate.py "$@" >> $O/c4am.log 2>&1 || exit 2
ABL_CONFIG=C5 ABL_DOCS=100000 timeout -k 10 300 python tools/ablate.py "$@" >> $O/c5.log 2>&1 || exit 3
timeout -k 10 300 python tools/ablate.py "$@" >> $O/c4.log 2>&1 || exit 1
cat $O/c4am.log $O/c5.log $O/c4.log
