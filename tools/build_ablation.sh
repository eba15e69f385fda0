#!/bin/bash
# Diagnostic builds of libzp with conv / wgrad ablations (ZP_ABL=1: no LDS-DMA in the loop, 2: no
# MFMA, 3: weights only, 4: strips only, 5: no epilogue (k_conv_quad); results are wrong): zebrapose_amd/libzp_abl<N>.so.  Only
# zp_conv.hip is rebuilt; the other objects come from the product build (make first).
# Use with ZP_LIB=zebrapose_amd/libzp_abl<N>.so python tools/conv_ab.py ...
set -e
cd "$(dirname "$0")/../zebrapose_amd/csrc"
for n in "$@"; do
  mkdir -p build_abl$n
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DZP_ABL=$n -c zp_conv.hip -o build_abl$n/zp_conv.o &
done
wait
for n in "$@"; do
  objs=$(ls build/*.o | grep -v zp_conv.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../libzp_abl$n.so build_abl$n/zp_conv.o $objs
done
