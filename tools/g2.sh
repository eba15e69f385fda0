set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > gpurun_out/g2_bench.json 2> gpurun_out/g2_bench.err
echo "bench rc $?"
NO_TRAIN=1 bash tools/prof_r03.sh r03a > gpurun_out/g2_prof.log 2>&1
echo "prof rc $?"
