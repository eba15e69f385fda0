set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
P="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for m in 0 2; do
timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/g15_pmc$m -o run -- python3 tools/conv3_ab.py --strip $m --flags 478 --layers up2conv,up1conv --rounds 1 --iters 2 > gpurun_out/g15_pmc$m.log 2>&1; chk $? pmc$m
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/g15_l2$m -o run -- python3 tools/conv3_ab.py --strip $m --flags 478 --layers up2conv,up1conv --rounds 1 --iters 2 > gpurun_out/g15_l2$m.log 2>&1; chk $? l2$m
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_v3.py -q -s -k "bf16" --timeout 250 --timeout-method thread > gpurun_out/g15_bands.log 2>&1; chk $? bands
