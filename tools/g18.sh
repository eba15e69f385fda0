set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py -q -s -x --timeout 200 --timeout-method thread > gpurun_out/g18_x3.log 2>&1; chk $? x3
timeout -k 10 300 python -u tools/conv3_ab.py --form h2 --flags 478 --layers up2conv,l5,up2T,up1conv,l2,l1 > gpurun_out/g18_ab_h2.log 2>&1; chk $? abh2
timeout -k 10 300 python -u tools/conv3_ab.py --form x3 --flags 478 --layers up2conv,l5,up2T,up1conv,l2,l1 > gpurun_out/g18_ab_x3.log 2>&1; chk $? abx3
timeout -k 10 300 python -u tools/x3_accuracy.py > gpurun_out/g18_acc.log 2>&1; chk $? acc
