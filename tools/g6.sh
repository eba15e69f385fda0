set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/x3_accuracy.py > gpurun_out/g6_acc.log 2>&1
echo "acc rc $?"
