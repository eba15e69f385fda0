set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
timeout -k 10 400 python -u tools/conv3_ab.py --form h2 --flags 478,262622 --layers up2T,up1T > gpurun_out/g38_ab.log 2>&1; chk $? ab
