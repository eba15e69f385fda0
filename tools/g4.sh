set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_x3.py -v -s --timeout 200 --timeout-method thread > gpurun_out/g4_pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_geometry.py -k "fp32" -v -s --timeout 250 --timeout-method thread > gpurun_out/g4_pytest_bg.log 2>&1
echo "pytest bg rc $?"
