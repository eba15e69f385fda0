set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_pnp.py tests/test_gpu_multi_object.py tests/test_gpu_parity.py -q --timeout 250 --timeout-method thread > gpurun_out/g26_t.log 2>&1; chk $? tests
timeout -k 10 400 python -u bench.py > gpurun_out/g26_bench.log 2>&1; chk $? bench
