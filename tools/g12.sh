set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py -q --timeout 200 --timeout-method thread > gpurun_out/g12_x3.log 2>&1; chk $? x3
timeout -k 10 300 python -u tools/conv3_ab.py --flags 478,470,4574,8670 --layers up2conv,l5,up2T,up1conv > gpurun_out/g12_ab0.log 2>&1; chk $? ab0
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/g12_l2 -o run -- python3 tools/conv3_ab.py --flags 478 --layers up2conv,l5 --rounds 1 --iters 2 > gpurun_out/g12_l2.log 2>&1; chk $? l2
