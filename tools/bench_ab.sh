#!/bin/bash
# Same-box A/B of conv schedule flags on the whole inference step (bench.py, inference leg only),
# alternating variants: bash tools/bench_ab.sh "222 478" [rounds]
set -e
V=${1:-"222 478"}
R=${2:-2}
for r in $(seq $R); do
  for f in $V; do
    out=$(ZP_CONV_FLAGS=$f timeout -k 10 120 python3 bench.py --no-train --no-cpu --no-multi --no-bf16 --steps 20 --warmup 5 2>/dev/null | tail -1)
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); r=d['roofline']; print('flags', sys.argv[1], 'crops/s', d['value'], 'frac', r['frac'], 'avg_us', r['avg_launch_us'])" $f "$out"
  done
done
