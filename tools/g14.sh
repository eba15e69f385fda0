set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py -q -s --timeout 200 --timeout-method thread > gpurun_out/g14_x3.log 2>&1; chk $? x3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g14_all.log 2>&1; chk $? all
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/g14_pmc -o run -- python3 tools/conv3_ab.py --flags 478 --layers up2conv,up1conv,l1 --rounds 1 --iters 2 > gpurun_out/g14_pmc.log 2>&1; chk $? pmc
