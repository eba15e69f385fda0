set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_geometry.py tests/test_gpu_graphs.py -q -s --timeout 300 --timeout-method thread > gpurun_out/g31_t.log 2>&1; chk $? tests
timeout -k 10 300 python -u tools/x3_accuracy.py > gpurun_out/g31_acc.log 2>&1; chk $? acc
timeout -k 10 400 python -u bench.py --no-train --no-multi --no-cpu > gpurun_out/g31_bench.log 2>&1; chk $? bench
