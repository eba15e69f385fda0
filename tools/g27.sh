set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
timeout -k 10 400 python -u tools/bs1_engines.py > gpurun_out/g27_bs1.log 2>&1; chk $? bs1
