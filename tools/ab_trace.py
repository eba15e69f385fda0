"""Per-setting average kernel durations from a rocprofv3 kernel trace of tools/conv3_ab.py:
python scratch/ab_trace.py <trace.csv> <kernel substring> <n settings> <n layers> <iters> <rounds>"""
import csv, sys
path, sub, nset, nlay, iters, rounds = sys.argv[1], sys.argv[2], *map(int, sys.argv[3:7])
rows = [r for r in csv.DictReader(open(path)) if sub in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Dispatch_Id"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows]
per = (2 + iters)
print(len(d), "dispatches; expected", rounds * nset * nlay * per)
res = {}
k = 0
for r in range(rounds):
    for s in range(nset):
        for l in range(nlay):
            blk = d[k:k + per]; k += per
            res.setdefault((s, l), []).append(sum(blk[2:]) / iters)
for (s, l), v in sorted(res.items()):
    print(f"setting {s} layer {l}: min {min(v):.1f} us  all {[round(x,1) for x in v]}")
