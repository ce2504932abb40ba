#!/bin/bash
# Build A/B variants of libhmgpu.so for tools/ablate.py: tools/build_variants.sh name:"-DFLAG=1 ..." ...
#   -> hypermerge_amd/_lib/ablate/lib_<name>.so   (dev tool; the product build is hypermerge_amd/build.py)
cd "$(dirname "$0")/../hypermerge_amd/_lib" && mkdir -p ablate && cd ablate
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -mllvm -amdgpu-atomic-optimizer-strategy=DPP $flags -o lib_$name.so \
    ../../csrc/merge_kernels.hip ../../csrc/merge_large.hip ../../csrc/store_kernels.hip ../../csrc/engine.cpp ../../csrc/store.cpp &
done
wait
ls
