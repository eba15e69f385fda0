set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 250 --timeout-method thread > gpurun_out/g10_pytest.log 2>&1; chk $? pytest
