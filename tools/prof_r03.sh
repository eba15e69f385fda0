#!/bin/bash
# Runs on the GPU box (gpurun).  Round-3 profile set, every rocprofv3 run its own process and time
# limit, PMC passes separate from the traces (and never combined with a trace domain):
#   stats        kernel-trace --stats over bench.py's inference legs (fp32 headline + bf16 leg)
#   trace_<p>    per-dispatch kernel trace of tools/prof_driver.py --mode infer (precision p) + its
#                stage log (which network stage each conv launch belongs to)
#   fetch_<p> / write_<p> / mfma_<p>   PMC passes over the same driver run: FETCH_SIZE; WRITE_SIZE;
#                SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE + SQ_INSTS_VALU_MFMA_MOPS_{BF16,F32}
#   train_1s     kernel-trace --stats of the bs=32 bf16 training step on ONE stream
#                (ZP_SIDE_WGRAD=0: weight gradients not overlapped, so per-kernel durations attribute)
#   ttrace / tfetch / twrite (TRAIN_PMC=1, round 6)   kernel trace + FETCH_SIZE + WRITE_SIZE passes over
#                the same one-stream training step (tools/prof_train.py)
# Summarise with tools/prof_stages.py <tag>.
set -e -o pipefail
TAG=${1:-r03}
PRECS=${PRECS:-"fp32 bf16"}
O=gpurun_out/prof_$TAG
mkdir -p $O
export TMPDIR=/tmp
D="python3 tools/prof_driver.py --mode infer --steps 3 --warmup 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
    python3 bench.py --no-train --no-cpu --no-multi --no-bs1 --steps 10 --warmup 3 > $O/stats.log 2>&1
echo "stats ok"
for P in $PRECS; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$P -o run -- \
      $D --precision $P --stage-log $O/stage_log_$P.json > $O/trace_$P.log 2>&1
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$P -o run -- \
      $D --precision $P > $O/fetch_$P.log 2>&1
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$P -o run -- \
      $D --precision $P > $O/write_$P.log 2>&1
  timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 \
      SQ_INSTS_VALU_MFMA_MOPS_F32 --output-format csv -d $O/mfma_$P -o run -- \
      $D --precision $P > $O/mfma_$P.log 2>&1
  echo "$P ok"
done
if [ -z "$NO_TRAIN" ]; then
  ZP_SIDE_WGRAD=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/train_1s -o run -- \
      python3 tools/prof_driver.py --mode train --steps 5 --warmup 2 > $O/train_1s.log 2>&1
  echo "train ok"
fi
if [ -n "$TRAIN_PMC" ]; then  # round 6: counter passes over the training step (tools/prof_train.py)
  T="python3 tools/prof_driver.py --mode train --steps 3 --warmup 2"
  ZP_SIDE_WGRAD=0 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/ttrace -o run -- \
      $T --stage-log $O/stage_log_train.json > $O/ttrace.log 2>&1
  ZP_SIDE_WGRAD=0 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/tfetch -o run -- \
      $T > $O/tfetch.log 2>&1
  ZP_SIDE_WGRAD=0 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/twrite -o run -- \
      $T > $O/twrite.log 2>&1
  echo "train pmc ok"
fi
echo done
