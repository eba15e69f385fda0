#!/bin/bash
# Diagnostic builds of libzp with k_conv ablations (ZP_ABL=1: no LDS-DMA, 2: no MFMA; results are
# wrong): zebrapose_amd/libzp_abl<N>.so.  Use with ZP_LIB=... python tools/conv_micro.py.
set -e
cd "$(dirname "$0")/../zebrapose_amd/csrc"
for n in "$@"; do
  mkdir -p build_abl$n
  for f in *.hip; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DZP_ABL=$n -c $f -o build_abl$n/${f%.hip}.o &
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../libzp_abl$n.so build_abl$n/*.o
done
