#!/bin/bash
# k_conv_quad ablations (diagnostic ZP_ABL builds from tools/build_ablation.sh): product, no LDS-DMA
# in the loop (1), no epilogue (5), no output stores (6); up2 / up1 ConvTranspose2d shapes, bs 32.
set -e
L=T320:256:64,T256:256:32
for n in 0 1 5 6; do
  lib=zebrapose_amd/libzp.so; [ $n != 0 ] && lib=zebrapose_amd/libzp_abl$n.so
  echo "== ABL $n"
  ZP_LIB=$lib timeout -k 10 120 python tools/conv_ab.py --layers $L --flags 478 --rounds 5 --iters 10 2>&1 | grep flags
done
echo "== strip DMA in the read section (222) vs between step-0 MFMAs (478)"
timeout -k 10 200 python tools/conv_ab.py --layers $L --flags 222,478 --rounds 7 --iters 10 2>&1 | grep flags
