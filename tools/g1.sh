set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/g1_counters.txt 2>&1 || true
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/g1_pytest.log 2>&1
echo "pytest rc $?"
