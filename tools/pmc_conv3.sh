#!/bin/bash
# PMC passes (one counter group per pass; gfx950 slot limits) over one split-fp32 layer of
# tools/conv3_ab.py:  tools/pmc_conv3.sh OUT LAYER WIDE   -> OUT/{sq,tcc,fetch,write}; read with tools/pmc_read.py
set -e -o pipefail
O=$1; LAYER=${2:-up2conv}; WIDE=${3:-1}
mkdir -p $O
export TMPDIR=/tmp
RUN="python3 tools/conv3_ab.py --form h2 --wide $WIDE --layers $LAYER --rounds 1 --iters 3"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $O/sq -o run -- $RUN > $O/sq.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/sq2 -o run -- $RUN > $O/sq2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/tcc -o run -- $RUN > $O/tcc.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- $RUN > $O/fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o run -- $RUN > $O/write.log 2>&1
echo done
