set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc $rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py -q -s -k "split_k" --timeout 250 --timeout-method thread > gpurun_out/g39_x3.log 2>&1; chk $? x3
timeout -k 10 400 python -u tools/bs1_engines.py > gpurun_out/g39_bs1.log 2>&1; chk $? bs1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g39_all.log 2>&1; chk $? all
