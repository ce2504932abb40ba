#!/bin/bash
# Build ablation variants of libhmgpu.so: tools/build_ablate.sh 0 64 ...  -> hypermerge_amd/_lib/ablate/lib_aNNN.so
cd "$(dirname "$0")/../hypermerge_amd/_lib" && mkdir -p ablate && cd ablate && rm -f lib_a*.so
for v in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -mllvm -amdgpu-atomic-optimizer-strategy=DPP -DHM_ABLATE=$v -o lib_a$(printf %03d $v).so \
    ../../csrc/merge_kernels.hip ../../csrc/merge_large.hip ../../csrc/store_kernels.hip ../../csrc/engine.cpp ../../csrc/store.cpp &
done
wait
ls
