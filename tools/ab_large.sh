#!/bin/bash
# A/B of merge_large_kernel builds on C3 (and C1 actor-major): stamps shares + bench lines per library.
# Usage: tools/ab_large.sh name...   (libraries hypermerge_amd/_lib/ablate/lib_<name>.so; "base" = default build)
set -o pipefail
mkdir -p gpurun_out
for nm in "$@"; do
  so=hypermerge_amd/_lib/ablate/lib_$nm.so; [ "$nm" = base ] && so=hypermerge_amd/_lib/libhmgpu.so
  if [ -f hypermerge_amd/_lib/ablate/lib_stamps_$nm.so ]; then
    HMGPU_LIB=hypermerge_amd/_lib/ablate/lib_stamps_$nm.so timeout -k 10 200 python tools/lstamps.py C3 10000 > gpurun_out/lstamps_$nm.log 2>&1 || exit 2
    echo "== stamps $nm"; cat gpurun_out/lstamps_$nm.log | grep -v amdgpu.ids
  fi
  for cfg in "C3 --docs 10000" "C1 --docs 1 --arrival 1"; do
    HMGPU_LIB=$so timeout -k 10 300 python bench.py --config $cfg --check-docs 200 --steps 5 --warmup 2 --no-cpu --no-traffic > gpurun_out/ab_$nm.log 2>&1 || { tail -5 gpurun_out/ab_$nm.log; exit 3; }
    tail -1 gpurun_out/ab_$nm.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$nm', '$cfg'.split()[0], 'value %.3e ms %.3f kernel_ms %.3f parity %s unsup %s' % (d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['parity_sample_ok'], d['unsupported_docs']))"
  done
done
