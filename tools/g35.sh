set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py -q -k "strip" --timeout 250 --timeout-method thread > gpurun_out/g35_x3.log 2>&1; chk $? x3
timeout -k 10 400 python -u tools/conv3_ab.py --form h2 --strip 0,1,2 --flags 478 --layers up2conv,up1conv,l4,l2,l1 > gpurun_out/g35_ab.log 2>&1; chk $? ab
