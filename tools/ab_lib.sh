#!/bin/bash
# Same-box A/B of two builds of libzp on given conv layers (tools/conv_ab.py through ZP_LIB),
# alternating: bash tools/ab_lib.sh <libA.so> <libB.so> [layers] [rounds]
# (e.g. a copy of the previous build against the current one; layers as tools/conv_ab.py takes them)
set -e
A=${1:?libA}
B=${2:?libB}
L=${3:-T320:256:64,T256:256:32}
R=${4:-2}
for r in $(seq $R); do
  for lib in $A $B; do
    echo "== $lib"
    ZP_LIB=$lib timeout -k 10 120 python tools/conv_ab.py --layers $L --flags 478 --rounds 5 --iters 10 2>&1 | grep flags
  done
done
