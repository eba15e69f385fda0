set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_parity.py tests/test_gpu_bench_geometry.py tests/test_gpu_v3.py -q --timeout 250 --timeout-method thread > gpurun_out/g17_t.log 2>&1; chk $? tests
timeout -k 10 300 python -u bench.py --no-train --no-multi --no-bs1 > gpurun_out/g17_bench.log 2>&1; chk $? bench
