#!/bin/bash
# Build A/B variants of libhmgpu.so for tools/ablate.py: tools/build_variants.sh name:"-DFLAG=1 ..." ...
#   -> hypermerge_amd/_lib/ablate/lib_<name>.so   (dev tool; the product build is hypermerge_amd/build.py)
# CSRC=<dir> builds from another source tree (e.g. a `git worktree` of an older commit).
R="$(cd "$(dirname "$0")/.." && pwd)"
SRC="${CSRC:-$R/hypermerge_amd/csrc}"
mkdir -p "$R/hypermerge_amd/_lib/ablate" && cd "$R/hypermerge_amd/_lib/ablate"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -mllvm -amdgpu-atomic-optimizer-strategy=DPP $flags -o lib_$name.so \
    $SRC/merge_kernels.hip $SRC/merge_large.hip $SRC/store_kernels.hip $SRC/inc_kernels.hip $SRC/exchange.hip $SRC/cursors.hip $SRC/engine.cpp $SRC/store.cpp $SRC/decode.cpp $SRC/docset.cpp -ldl &
done
wait
ls
