#!/bin/bash
# A/B of incremental-kernel variants (tools/build_variants.sh libs): the resident C4 rounds of
# tools/inc_profile.py under each library, the per-round incremental phase times.
set -o pipefail
O=gpurun_out/${1:-ab_inc}
shift
mkdir -p $O
for lib in "$@"; do
  for rep in 1 2; do
    HMGPU_LIB=$lib timeout -k 10 200 python tools/inc_profile.py --incremental 1 --device 1 > $O/$(basename $lib .so)_$rep.log 2>&1 || exit 1
    echo "$(basename $lib) $rep: $(grep -E '^\[hm_store\] incremental' $O/$(basename $lib .so)_$rep.log | awk '{print $3}' | tr '\n' ' ')"
  done
done
