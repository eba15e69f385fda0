set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_parity.py -k "split or fp32" -x -v --timeout 200 --timeout-method thread > gpurun_out/g3_pytest.log 2>&1
echo "pytest rc $?"
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_geometry.py -k "fp32" -x -v --timeout 250 --timeout-method thread > gpurun_out/g3_pytest_bg.log 2>&1
echo "pytest bg rc $?"
timeout -k 10 300 python3 bench.py --no-train --no-cpu --no-multi --no-bs1 --layer-report gpurun_out/g3_layers.json > gpurun_out/g3_bench.json 2> gpurun_out/g3_bench.err
echo "bench rc $?"
