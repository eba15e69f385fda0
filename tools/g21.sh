set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
timeout -k 10 300 python -u tools/h2_head_debug.py h2 x3 > gpurun_out/g21_dbg.log 2>&1; chk $? dbg
