set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_geometry.py -k "fp32_bench" -v -s --timeout 250 --timeout-method thread > gpurun_out/g5_pytest_bg.log 2>&1
rc=$?; echo "pytest bg rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/conv3_ab.py --flags 478,470,4574,8670,16862 --layers up2conv,l5,up2T > gpurun_out/g5_ab.log 2>&1
echo "ab rc $?"
