#!/bin/bash
# PMC of one weight-gradient launch (tools/conv_micro.py --wgrad).  Usage: tools/pmc_wgrad.sh <tag> <cin> <cout> <hw> <d>
set -e -o pipefail
TAG=$1; CI=$2; CO=$3; HW=$4; D=$5
O=gpurun_out/pmc_$TAG
mkdir -p $O
export TMPDIR=/tmp
run() {
  local n=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/$n -o run -- \
    python3 tools/conv_micro.py --wgrad --cin $CI --cout $CO --hw $HW --d $D --iters 3 > $O/$n.log 2>&1
}
run sq1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT
run sq2 SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAVES
echo done
