#!/usr/bin/env python3
"""Counter evidence for the training leg from a tools/prof_r03.sh run with the
train passes (gpurun_out/prof_<tag>/ttrace, tfetch, twrite, stage_log_train.json) ->
profiles/<tag>_train_pmc_traffic.json, keyed to the libzp.so build (lib_sha16) that bench.py reads
for train.roofline.traffic.

All three passes run the same program, tools/prof_driver.py --mode train (configs[2]: R34 bs=32
bf16, forward + hist-weighted BCE / mask loss + backward + Adam) on ONE stream (ZP_SIDE_WGRAD=0, so
every dispatch's duration is its own), whose dispatch sequence repeats per step.  The step window is
the last step: from its input conversion (k_nchw_to_nhwc, the first kernel of a forward) to the end
of the run.  Every kernel of the window counts toward the step, torch's own (fills, copies) too.

Per kernel label (tools/prof_summary.py bench_label; the weight-gradient kernels k_wgrad2 /
k_wgrad_lds / k_wgrad_reduce are one engine launch, 'k_wgrad+reduce'):
  launches      per step (engine launches: the stage log's count for the label)
  us            kernel-trace durations
  read / write  2 x FETCH_SIZE x 1024 B, WRITE_SIZE x 1024 B (MI355X_MICROARCH.md HBM section)
  algorithmic   the engine's per-launch algorithmic bytes (inputs, packed weights and outputs read /
                written once; stage_log_train.json) and FLOPs
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from prof_summary import bench_label  # noqa: E402


def one(pattern):
    f = sorted(glob.glob(pattern, recursive=True))
    return f[0] if f else None


def label(name):
    lab = bench_label(name)
    if lab:
        return lab
    if "k_wgrad" in name:  # k_wgrad2 / k_wgrad_lds / k_wgrad_reduce: one engine launch
        return "k_wgrad+reduce"
    return name.split("(")[0].replace("void ", "")


def last_window(rows):
    starts = [i for i, r in enumerate(rows) if "k_nchw_to_nhwc" in r[0]]
    if not starts:
        raise SystemExit("no k_nchw_to_nhwc dispatch (training forward start) found")
    return rows[starts[-1]:]


def read_trace(path):
    out = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            out.append((r["Kernel_Name"], int(r["Dispatch_Id"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    return sorted(out, key=lambda t: t[1])


def read_pmc(path, counter):
    per, kn = defaultdict(float), {}
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if r["Counter_Name"] != counter:
                continue
            d = int(r["Dispatch_Id"])
            per[d] += float(r["Counter_Value"])
            kn[d] = r["Kernel_Name"]
    return [(kn[d], d, per[d]) for d in sorted(per)]


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    log = json.load(open(os.path.join(src, "stage_log_train.json")))
    tr = last_window(read_trace(one(os.path.join(src, "ttrace", "**", "*kernel_trace.csv"))))
    fe = last_window(read_pmc(one(os.path.join(src, "tfetch", "**", "*counter_collection.csv")), "FETCH_SIZE"))
    wr = last_window(read_pmc(one(os.path.join(src, "twrite", "**", "*counter_collection.csv")), "WRITE_SIZE"))
    if not (len(tr) == len(fe) == len(wr)):
        raise SystemExit(f"step windows differ: trace {len(tr)} fetch {len(fe)} write {len(wr)}")
    for a, b, c in zip(tr, fe, wr):
        if not (a[0] == b[0] == c[0]):
            raise SystemExit(f"dispatch sequences differ between passes: {a[0][:60]} / {b[0][:60]} / {c[0][:60]}")
    agg = defaultdict(lambda: defaultdict(float))
    step = defaultdict(float)
    for (name, _, ns), f, w in zip(tr, fe, wr):
        lab = label(name)
        rd, wb = 2.0 * 1024.0 * f[2], 1024.0 * w[2]
        d = agg[lab]
        d["dispatches"] += 1
        d["ns"] += ns
        d["read"] += rd
        d["write"] += wb
        step["dispatches"] += 1
        step["ns"] += ns
        step["read"] += rd
        step["write"] += wb
    eng = log["kernels"]
    by = {}
    for lab, d in agg.items():
        e = eng.get(lab)
        n = int(e["launches"]) if e else int(d["dispatches"])
        row = {"dispatches_per_step": int(d["dispatches"]), "launches_per_step": n,
               "us_per_step": round(d["ns"] / 1e3, 1), "us_per_launch": round(d["ns"] / 1e3 / n, 2),
               "read_bytes_per_launch": round(d["read"] / n), "write_bytes_per_launch": round(d["write"] / n),
               "hbm_bytes_per_launch": round((d["read"] + d["write"]) / n)}
        if e and e["bytes"]:
            row["algorithmic_bytes_per_launch"] = round(e["bytes"] / n)
            row["traffic_over_algorithmic"] = round((d["read"] + d["write"]) / e["bytes"], 3)
        if e and e["flops"]:
            row["algorithmic_flop_per_launch"] = round(e["flops"] / n)
            row["tflops"] = round(e["flops"] / d["ns"] / 1e3, 1)
            row["frac_of_bf16_peak"] = round(e["flops"] / d["ns"] / 1e3 / 2516.6, 4)
        by[lab] = row
    out = {"source": "tools/prof_r03.sh train passes: rocprofv3 --kernel-trace / --pmc FETCH_SIZE / --pmc WRITE_SIZE "
                     "(separate runs) over ZP_SIDE_WGRAD=0 python3 tools/prof_driver.py --mode train --steps 3 "
                     "--warmup 2 (one stream), the last step",
           "correction": "bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 (MI355X_MICROARCH.md HBM section)",
           "lib_sha16": log["lib_sha16"], "batch": log["batch"], "precision": log["precision"],
           "step": {"dispatches": int(step["dispatches"]), "kernel_us": round(step["ns"] / 1e3, 1),
                    "read_bytes": round(step["read"]), "write_bytes": round(step["write"]),
                    "hbm_bytes": round(step["read"] + step["write"]),
                    "hbm_gbps_over_kernel_time": round((step["read"] + step["write"]) / step["ns"], 1)},
           "by_label": dict(sorted(by.items(), key=lambda kv: -kv[1]["us_per_step"]))}
    dst = os.path.join(ROOT, "profiles", f"{tag}_train_pmc_traffic.json")
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(f"== {dst}: step {out['step']}")
    for lab, r in list(out["by_label"].items())[:15]:
        print(f"{r['us_per_step']:9.1f} us  {r['launches_per_step']:4d} x  {r['hbm_bytes_per_launch'] / 1e6:8.2f} MB"
              f"  (algo {r.get('algorithmic_bytes_per_launch', 0) / 1e6:8.2f})  {r.get('tflops')} TF  {lab}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r06")
