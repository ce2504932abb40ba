#!/bin/bash
# Profile bench.py's dominant kernel on the GPU box (run via gpurun from the repo root).
#   pass 0: kernel trace + stats (durations)
#   pass 1: SQ wave-state counters
#   pass 2: FETCH_SIZE         pass 3: WRITE_SIZE   (separate passes: TCC slot limits)
# Usage: tools/profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-prof}; shift
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
ARGS="--steps 3 --warmup 1 --no-cpu --no-traffic --no-e2e --no-orders --no-incremental --no-node --check-docs 0 $*"
# the trace pass times more steps, so its per-kernel average is the warm steady state the bench
# line's HIP events report (the first launch after the host's setup meets a down-clocked GPU)
TARGS="--steps 20 --warmup 3 --no-cpu --no-traffic --no-e2e --no-orders --no-incremental --no-node --check-docs 0 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $TARGS > $OUT/trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $OUT/pmc1 -o run -- python3 $R/bench.py $ARGS > $OUT/pmc1.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc2 -o run -- python3 $R/bench.py $ARGS > $OUT/pmc2.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc3 -o run -- python3 $R/bench.py $ARGS > $OUT/pmc3.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc4 -o run -- python3 $R/bench.py $ARGS > $OUT/pmc4.log 2>&1 || exit 5
echo done
