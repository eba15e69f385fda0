#!/bin/bash
# Runs on the GPU box (gpurun): kernel-trace stats for inference and training, then the two PMC
# passes (FETCH_SIZE, WRITE_SIZE -- separate runs, TCC slots) over the inference step, then the same
# two passes over the training step.
# Output under gpurun_out/prof_<tag>/ ; summarise with tools/prof_summary.py.
set -e -o pipefail
TAG=${1:-r02}
O=gpurun_out/prof_$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/infer -o run -- \
    python3 bench.py --no-train --no-cpu --no-multi --no-bf16 --no-bs1 --steps 10 --warmup 3 > $O/infer.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/train -o run -- \
    python3 tools/prof_driver.py --mode train --steps 5 --warmup 2 > $O/train.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- \
    python3 tools/prof_driver.py --mode infer --steps 3 --warmup 1 > $O/pmc_fetch.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- \
    python3 tools/prof_driver.py --mode infer --steps 3 --warmup 1 > $O/pmc_write.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/tpmc_fetch -o run -- \
    python3 tools/prof_driver.py --mode train --steps 2 --warmup 1 > $O/tpmc_fetch.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/tpmc_write -o run -- \
    python3 tools/prof_driver.py --mode train --steps 2 --warmup 1 > $O/tpmc_write.log 2>&1
echo done
