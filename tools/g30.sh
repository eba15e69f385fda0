set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
timeout -k 10 400 python -u tools/conv3_ab.py --form h2 --flags 478,131550,470,131542 --layers up2conv,l5,up1conv,l4,up2T > gpurun_out/g30_ab.log 2>&1; chk $? ab
