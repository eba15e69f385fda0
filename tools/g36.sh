set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_tf.py tests/test_gpu_parity.py tests/test_gpu_units.py tests/test_gpu_v3.py tests/test_gpu_rccl.py -q -x --timeout 300 --timeout-method thread > gpurun_out/g36_t.log 2>&1; chk $? tests
ZP_SIDE_WGRAD=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g36_train -o run -- python3 tools/prof_driver.py --mode train --steps 5 --warmup 2 > gpurun_out/g36_train.log 2>&1; chk $? train
timeout -k 10 300 python3 tools/prof_driver.py --mode train --steps 10 --warmup 3 > gpurun_out/g36_train_time.log 2>&1; chk $? traintime
