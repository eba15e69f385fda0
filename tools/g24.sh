set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
timeout -k 10 300 python -u tools/conv3_ab.py --form h2 --flags 478,33246,470,482 --layers up2conv,l5,up2T,up1conv,l4 > gpurun_out/g24_ab.log 2>&1; chk $? ab
timeout -k 10 300 python -u tools/conv3_ab.py --form h2 --strip 2 --flags 478 --layers up2conv,up1conv,l4,l2,l1 > gpurun_out/g24_ab_s2.log 2>&1; chk $? abs2
timeout -k 10 300 python -u tools/conv3_ab.py --form h2 --strip 0 --flags 478 --layers up2conv,up1conv,l4,l2,l1 > gpurun_out/g24_ab_s0.log 2>&1; chk $? abs0
