set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
timeout -k 10 300 python -u tools/conv3_ab.py --flags 478 --minblocks 0,256,512,1024 --layers l2,l4,l5,up1conv > gpurun_out/g16_ab.log 2>&1; chk $? ab
