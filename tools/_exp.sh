export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 5 150 python bench.py --no-cpu --layer-report gpurun_out/il.json > gpurun_out/b.log 2>&1 || exit 1
