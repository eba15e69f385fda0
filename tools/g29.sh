set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
P="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/g29_pmc -o run -- python3 tools/conv3_ab.py --form h2 --flags 478 --layers up2conv,l5 --rounds 1 --iters 2 > gpurun_out/g29_pmc.log 2>&1; chk $? pmc
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/g29_l2 -o run -- python3 tools/conv3_ab.py --form h2 --flags 478 --layers up2conv,l5 --rounds 1 --iters 2 > gpurun_out/g29_l2.log 2>&1; chk $? l2
