#!/bin/bash
# Diagnostic library: libzp with the wide tile's per-segment clock stamps (zp_conv3w.hip, ZP_STAMP),
# loaded through ZP_LIB=tools/stamp/libzp_stamp.so by tools/stamp_conv3w.py.  The product objects of
# the other sources are reused (zebrapose_amd/csrc/build, from `make`); only zp_conv3w.hip is rebuilt.
set -euo pipefail
cd "$(dirname "$0")/.."
make -C zebrapose_amd/csrc -j8 >/dev/null
mkdir -p tools/stamp/build
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-variable \
  -fno-slp-vectorize -DZP_STAMP -c zebrapose_amd/csrc/zp_conv3w.hip -o tools/stamp/build/zp_conv3w.o
objs=$(ls zebrapose_amd/csrc/build/*.o | grep -v '/zp_conv3w.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/stamp/libzp_stamp.so $objs tools/stamp/build/zp_conv3w.o
echo "built tools/stamp/libzp_stamp.so"
