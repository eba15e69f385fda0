#!/bin/bash
# PMC passes over the eval inference step (one pass per counter group; gfx950 slot limits).
set -e -o pipefail
O=gpurun_out/pmc_conv
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $O/sq -o run -- python3 tools/prof_driver.py --mode infer --steps 2 --warmup 1 > $O/sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/tcc -o run -- python3 tools/prof_driver.py --mode infer --steps 2 --warmup 1 > $O/tcc.log 2>&1
echo done
