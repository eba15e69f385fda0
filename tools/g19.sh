set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
timeout -k 10 300 python -u tools/h2_debug.py > gpurun_out/g19_dbg.log 2>&1; chk $? dbg
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py -q -s --timeout 200 --timeout-method thread > gpurun_out/g19_x3.log 2>&1; chk $? x3
