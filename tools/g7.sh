set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py -q -x --timeout 200 --timeout-method thread > gpurun_out/g7_x3.log 2>&1; chk $? x3
timeout -k 10 300 python -u tools/x3_accuracy.py > gpurun_out/g7_acc.log 2>&1; chk $? acc
timeout -k 10 300 python -u tools/conv3_ab.py --flags 470,4566,8662 --layers up2conv,l5,up2T,up1conv,l1 > gpurun_out/g7_ab0.log 2>&1; chk $? ab0
ZP_CONV3_SCHED=1 timeout -k 10 300 python -u tools/conv3_ab.py --flags 470 --layers up2conv,l5,up2T > gpurun_out/g7_ab1.log 2>&1; chk $? ab1
timeout -k 10 300 python3 bench.py --no-train --no-cpu --no-multi --no-bs1 --no-bf16 --layer-report gpurun_out/g7_layers.json > gpurun_out/g7_bench.json 2> gpurun_out/g7_bench.err; chk $? bench
