set -e
L=256:256:128:1,512:512:32:4,256:256:64:1
for n in 0 8 6; do
  lib=zebrapose_amd/libzp.so; [ $n != 0 ] && lib=zebrapose_amd/libzp_abl$n.so
  echo "== ABL $n"
  ZP_LIB=$lib timeout -k 10 120 python tools/conv_ab.py --layers $L --flags 478 --rounds 5 --iters 10 2>&1 | grep flags
done
