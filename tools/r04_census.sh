#!/bin/bash
# round 4: the C5 resident rounds' append census (HM_STORE_PROFILE) and phase marks
set -o pipefail
O=gpurun_out/r04/census
mkdir -p $O
timeout -k 10 240 python tools/inc_profile.py --config C5 --docs 100000 --device 1 --incremental 0 > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
timeout -k 10 240 python tools/inc_profile.py --config C4 --docs 1000000 --device 1 --incremental 0 > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 1; }
grep -h "append\|round" $O/c5.log $O/c4.log
