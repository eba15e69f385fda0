set -e
L=T320:256:64,T256:256:32
for r in 1 2; do
for lib in zebrapose_amd/libzp_abl9.so zebrapose_amd/libzp.so; do
  echo "== $lib"
  ZP_LIB=$lib timeout -k 10 120 python tools/conv_ab.py --layers $L --flags 478 --rounds 5 --iters 10 2>&1 | grep flags
done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_units.py -q -k "quad" --timeout 300 --timeout-method thread 2>&1 | tail -2
