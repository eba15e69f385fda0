#!/usr/bin/env python3
"""Print per-dispatch averages of every counter of a tools/pmc_layer.sh run (conv kernels only)."""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
vals = defaultdict(list)
for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if "k_conv" not in r["Kernel_Name"] and "k_wgrad" not in r["Kernel_Name"]:
            continue
        vals[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(vals.items()):
    print(f"{c:32s} {sum(v) / len(v):16.1f}   n={len(v)}  {k}")
