set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py -q --timeout 200 --timeout-method thread > gpurun_out/g13_x3.log 2>&1; chk $? x3
ZP_CONV3_STRIP=0 timeout -k 10 200 python -u tools/conv3_ab.py --flags 478 --layers up2conv,up1conv,l1 > gpurun_out/g13_ab_s0.log 2>&1; chk $? ab0
ZP_CONV3_STRIP=1 timeout -k 10 200 python -u tools/conv3_ab.py --flags 478,470 --layers up2conv,up1conv,l1 > gpurun_out/g13_ab_s1.log 2>&1; chk $? ab1
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_geometry.py -q -k "split_f32" --timeout 300 --timeout-method thread -s > gpurun_out/g13_geo.log 2>&1; chk $? geo
timeout -k 10 300 python -u tools/x3_accuracy.py > gpurun_out/g13_acc.log 2>&1; chk $? acc
timeout -k 10 300 python -u bench.py > gpurun_out/g13_bench.log 2>&1; chk $? bench
