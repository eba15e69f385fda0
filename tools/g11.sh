set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl.py tests/test_dist_buckets.py -m gpu -v --timeout 250 --timeout-method thread > gpurun_out/g11_pytest.log 2>&1; chk $? pytest
