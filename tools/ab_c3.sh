#!/bin/bash
# A/B of merge_large_kernel variants on C3 (and C1 actor-major): tools/ab_c3.sh <out> <variant>...
# variant "base" = the product library; others = hypermerge_amd/_lib/ablate/lib_<v>.so (tools/build_variants.sh)
OUT=$1; shift
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
for v in "$@"; do
  if [ "$v" = base ]; then unset HMGPU_LIB; else export HMGPU_LIB=$PWD/hypermerge_amd/_lib/ablate/lib_$v.so; fi
  for cfg in "C3 --docs 10000" "C1 --docs 1 --arrival 1"; do
    echo "== $v $cfg" >> "$OUT"
    timeout -k 10 240 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu --no-e2e --no-orders --no-traffic \
      --no-incremental --no-node --check-docs 100 >> "$OUT" 2>&1 || { echo "FAILED rc=$?" >> "$OUT"; exit 1; }
  done
done
