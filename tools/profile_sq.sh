#!/bin/bash
# Extra SQ stall-attribution passes for bench.py's dominant kernel (run via gpurun from the repo root).
# Usage: tools/profile_sq.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-prof}; shift
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
ARGS="--steps 3 --warmup 1 --no-cpu --no-traffic --no-e2e --no-orders --check-docs 0 $*"
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_IFETCH SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM --output-format csv -d $OUT/pmc5 -o run -- python3 $R/bench.py $ARGS > $OUT/pmc5.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_LDS_ATOMIC SQ_LDS_ATOMIC_RETURN SQ_IFETCH_LEVEL --output-format csv -d $OUT/pmc6 -o run -- python3 $R/bench.py $ARGS > $OUT/pmc6.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INSTS_VSKIPPED SQ_LEVEL_WAVES --output-format csv -d $OUT/pmc7 -o run -- python3 $R/bench.py $ARGS > $OUT/pmc7.log 2>&1 || exit 3
echo done
