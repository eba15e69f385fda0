#!/bin/bash
# PMC passes over one conv layer (tools/conv_ab.py, one variant), one rocprofv3 run per counter group
# (gfx950 slot limits: 8 SQ, 4 TCC, 2 GRBM per pass).  Usage: tools/pmc_layer.sh <tag> <layer> <flags>
set -e -o pipefail
TAG=${1:-l}; LAYER=${2:-256:256:128:1}; FLAGS=${3:-28}
O=gpurun_out/pmc_$TAG
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, counters...
  local n=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/$n -o run -- \
    python3 tools/conv_ab.py --layers $LAYER --flags $FLAGS --rounds 1 --iters 3 > $O/$n.log 2>&1
}
run sq1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT
run sq2 SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL
run sq3 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_LEVEL_LDS SQ_WAVES
run tcc TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
run fetch FETCH_SIZE
echo done
