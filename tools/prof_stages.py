#!/usr/bin/env python3
"""Per-stage MFMA utilisation and HBM traffic of the R34 inference step from a tools/prof_r03.sh run
(gpurun_out/prof_<tag>/) -> profiles/<tag>_stages_<precision>.json / .md, plus the per-kernel PMC
traffic file bench.py reads (profiles/<tag>_pmc_traffic.json, keyed to the libzp.so build hash) and
the kernel-trace stats (profiles/<tag>_infer_kernel_stats.csv, <tag>_train1s_kernel_stats.csv).

Attribution: every pass runs the same tools/prof_driver.py --mode infer program, whose dispatch
sequence is identical from step 2 on.  The last step is the window from its k_nchw_to_nhwc (the
input conversion, first kernel of a step; the two-plane engine's k_stem_h2, which reads the NCHW
input itself since round 5) to the end of the run (the decode kernels end it).  Its
conv dispatches are matched one by one, in order, to the driver's stage log (engine.stage_log:
stage, kernel label, FLOPs); the label of every pair is checked.  Non-conv kernels are attributed
by name (nchw_to_nhwc, im2col -> stem, maxpool -> layer1, global avgpool / broadcast -> aspp, decode).

Per stage:
  time      sum of the dispatch durations (kernel-trace pass, End - Start timestamps)
  TFLOP/s   algorithmic FLOPs (2 M taps Cin Cout per conv) / time; frac of the dtype's
            dense MFMA peak (bf16 2516.6, f32 157.3 TFLOP/s)
  MFMA busy SQ_VALU_MFMA_BUSY_CYCLES (per-SIMD busy cycles, summed) / (GRBM_GUI_ACTIVE / 8 x 1024
            SIMDs): the fraction of the stage's active cycles the matrix pipes were busy
            (rocprofv3's MfmaUtil formula; GRBM_GUI_ACTIVE is reported summed over the 8 XCDs;
            it reads high on dispatches shorter than ~0.3 ms, so short stages read low)
  HBM       reads 2 x FETCH_SIZE x 1024 B + writes WRITE_SIZE x 1024 B (MI355X_MICROARCH.md §HBM:
            FETCH_SIZE halves wide coalesced reads on gfx950), GB/s over the stage time
"""
import csv
import glob
import json
import os
import re
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from prof_summary import bench_label  # noqa: E402

PEAK = {"bf16": 2516.6, "fp32": 157.3}
# the fp32 eval forward runs the split-fp32 engine (six bf16 MFMA products per f32 MAC): its
# ceiling is the bf16 peak / 6; frac_of_peak for fp32 stays against the f32 MFMA peak (157.3)
PEAK_SPLIT = {"x3": 2516.6 / 6, "h2": 2516.6 / 3}  # three bf16 planes / two fp16 planes
STAGES = ["stem", "layer1", "layer2", "layer4", "layer5", "aspp", "up1", "up2", "head", "decode"]


def one(pattern):
    f = sorted(glob.glob(pattern, recursive=True))
    return f[0] if f else None


def nonconv_stage(name):
    if "nchw_to_nhwc" in name or "im2col" in name:
        return "stem"
    if "maxpool" in name:
        return "layer1"
    if "avgpool" in name or "broadcast" in name or "hw_reduce" in name:
        return "aspp"
    if "decode" in name or "threshold" in name or "scan" in name:
        return "decode"
    if "head_combine" in name:  # the fused 16-bit head's second launch
        return "up2"
    return None


def is_conv(name):
    return bench_label(name) is not None


def last_step(rows):
    """rows: dispatches in order [(name, ...)] -> the slice of the last step."""
    starts = [i for i, r in enumerate(rows) if "nchw_to_nhwc" in r[0]]
    if not starts:  # round 5: the two-plane stem reads the NCHW input itself (no conversion kernel)
        starts = [i for i, r in enumerate(rows) if "k_stem_h2" in r[0]]
    if not starts:
        raise SystemExit("no k_nchw_to_nhwc / k_stem_h2 dispatch found")
    return rows[starts[-1]:]


def read_trace(path):
    out = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if "zp::" not in r["Kernel_Name"]:
                continue
            out.append((r["Kernel_Name"], int(r["Dispatch_Id"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    out.sort(key=lambda t: t[1])
    return out


def read_pmc(path, names):
    per = defaultdict(dict)
    kn = {}
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if "zp::" not in r["Kernel_Name"] or r["Counter_Name"] not in names:
                continue
            d = int(r["Dispatch_Id"])
            per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            kn[d] = r["Kernel_Name"]
    return [(kn[d], d, per[d]) for d in sorted(per)]


def attribute(rows, log):
    """rows of the last step -> [(stage, row)], checking conv labels against the stage log."""
    out, ci = [], 0
    for r in rows:
        if is_conv(r[0]):
            if ci >= len(log):
                raise SystemExit("more conv dispatches than stage-log entries")
            ent = log[ci]
            lab = bench_label(r[0])
            if lab != ent["kernel"]:
                raise SystemExit(f"conv dispatch {ci}: rocprof {lab} vs stage log {ent['kernel']}")
            out.append((ent["stage"], r, ent))
            ci += 1
        else:
            out.append((nonconv_stage(r[0]) or "other", r, None))
    if ci != len(log):
        raise SystemExit(f"{ci} conv dispatches vs {len(log)} stage-log entries")
    return out


def stage_table(src, prec):
    log = json.load(open(os.path.join(src, f"stage_log_{prec}.json")))
    tr = last_step(read_trace(one(os.path.join(src, f"trace_{prec}", "**", "*kernel_trace.csv"))))
    fe = last_step(read_pmc(one(os.path.join(src, f"fetch_{prec}", "**", "*counter_collection.csv")),
                            {"FETCH_SIZE"}))
    wr = last_step(read_pmc(one(os.path.join(src, f"write_{prec}", "**", "*counter_collection.csv")),
                            {"WRITE_SIZE"}))
    mf = last_step(read_pmc(one(os.path.join(src, f"mfma_{prec}", "**", "*counter_collection.csv")),
                            {"SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_INSTS_VALU_MFMA_MOPS_BF16",
                             "SQ_INSTS_VALU_MFMA_MOPS_F32"}))
    if not (len(tr) == len(fe) == len(wr) == len(mf)):
        raise SystemExit(f"{prec}: step windows differ: trace {len(tr)} fetch {len(fe)} write {len(wr)} mfma {len(mf)}")
    for a, b, c, d in zip(tr, fe, wr, mf):
        if not (a[0] == b[0] == c[0] == d[0]):
            raise SystemExit(f"{prec}: dispatch sequences differ between passes: {a[0][:60]} / {b[0][:60]}")
    at = attribute(tr, log["launches"])
    st = {s: defaultdict(float) for s in STAGES + ["other"]}
    per_kernel = defaultdict(lambda: defaultdict(float))
    disp = []  # round 6: every conv dispatch of the step (traffic per launch against its algorithmic bytes)
    for (stage, t, ent), f, w, m in zip(at, fe, wr, mf):
        if ent is not None:
            rd, wb = 2.0 * 1024.0 * f[2].get("FETCH_SIZE", 0.0), 1024.0 * w[2].get("WRITE_SIZE", 0.0)
            g = m[2].get("GRBM_GUI_ACTIVE", 0.0)
            disp.append({"stage": stage, "kernel": ent["kernel"], "geo": ent.get("geo"), "us": round(t[2] / 1e3, 2),
                         "tflops": round(ent["flops"] / t[2] / 1e3, 1) if t[2] else None,
                         "read_mb": round(rd / 1e6, 2), "write_mb": round(wb / 1e6, 2),
                         "algo_mb": round(ent["bytes"] / 1e6, 2),
                         "traffic_over_algo": round((rd + wb) / ent["bytes"], 3) if ent["bytes"] else None,
                         "mfma_busy_pct": round(100.0 * m[2].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (g / 8.0 * 1024.0), 1)
                         if g else None})
        d = st[stage]
        d["dispatches"] += 1
        d["ns"] += t[2]
        d["flops"] += ent["flops"] if ent else 0.0
        d["algo_bytes"] += ent["bytes"] if ent else 0.0
        d["read"] += 2.0 * 1024.0 * f[2].get("FETCH_SIZE", 0.0)
        d["write"] += 1024.0 * w[2].get("WRITE_SIZE", 0.0)
        d["mfma_busy"] += m[2].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        d["grbm"] += m[2].get("GRBM_GUI_ACTIVE", 0.0)
        d["mops_bf16"] += m[2].get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0)
        d["mops_f32"] += m[2].get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0.0)
        k = per_kernel[bench_label(t[0]) or t[0].split("(")[0]]
        k["n"] += 1
        k["ns"] += t[2]
        k["read"] += 2.0 * 1024.0 * f[2].get("FETCH_SIZE", 0.0)
        k["write"] += 1024.0 * w[2].get("WRITE_SIZE", 0.0)
        k["flops"] += ent["flops"] if ent else 0.0
        k["mfma_busy"] += m[2].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        k["grbm"] += m[2].get("GRBM_GUI_ACTIVE", 0.0)
    rows = []
    labels = " ".join(per_kernel)
    form = "h2" if any(k in labels for k in ("k_conv3<h2", "k_conv3s<h2", "k_conv3w<h2", "k_conv3w_head<h2")) else (
        "x3" if "k_conv3<x3" in labels or "k_conv3s<x3" in labels else None)
    tot = defaultdict(float)
    for s in STAGES + ["other"]:
        d = st[s]
        if not d["dispatches"]:
            continue
        for k, v in d.items():
            tot[k] += v
        rows.append(summarise(s, d, prec, form))
    rows.append(summarise("total", tot, prec, form))
    kern = {k: {"launches": int(v["n"]), "us_per_launch": round(v["ns"] / v["n"] / 1e3, 2),
                "hbm_bytes_per_launch": round((v["read"] + v["write"]) / v["n"]),
                "read_bytes_per_launch": round(v["read"] / v["n"]), "write_bytes_per_launch": round(v["write"] / v["n"]),
                "tflops": round(v["flops"] / v["ns"] / 1e3, 1) if v["flops"] else None,
                "mfma_busy_pct": round(100.0 * v["mfma_busy"] / (v["grbm"] / 8.0 * 1024.0), 1) if v["grbm"] else None}
            for k, v in per_kernel.items()}
    return {"precision": prec, "batch": log["batch"], "lib_sha16": log["lib_sha16"], "stages": rows,
            "split_form": form, "kernels": kern, "dispatches": disp}


def summarise(name, d, prec, form=None):
    t = d["ns"] * 1e-9
    busy = 100.0 * d["mfma_busy"] / (d["grbm"] / 8.0 * 1024.0) if d["grbm"] else None
    return {"stage": name, "dispatches": int(d["dispatches"]), "us": round(d["ns"] / 1e3, 1),
            "gflop": round(d["flops"] / 1e9, 2),
            "tflops": round(d["flops"] / t / 1e12, 1) if t and d["flops"] else None,
            "frac_of_peak": round(d["flops"] / t / 1e12 / PEAK[prec], 3) if t and d["flops"] else None,
            "frac_of_split_ceiling": (round(d["flops"] / t / 1e12 / PEAK_SPLIT[form], 3)
                                      if form and t and d["flops"] else None),
            "mfma_busy_pct": None if busy is None else round(busy, 1),
            "hbm_mb": round((d["read"] + d["write"]) / 1e6, 1),
            "algo_mb": round(d["algo_bytes"] / 1e6, 1),
            "hbm_gbps": round((d["read"] + d["write"]) / t / 1e9, 1) if t else None,
            "mfma_mops_bf16": d["mops_bf16"], "mfma_mops_f32": d["mops_f32"]}


def md(tab):
    p = tab["precision"]
    form = tab.get("split_form")
    x3 = bool(form)
    peak = (f"frac of f32 MFMA peak 157.3 | frac of split ceiling {PEAK_SPLIT[form]:.1f}" if x3
            else "frac of bf16 peak 2516.6")
    eng = {"x3": " (split-fp32 engine, three bf16 planes)", "h2": " (split-fp32 engine, two fp16 planes)"}.get(form, "")
    out = [f"### R34 inference bs={tab['batch']}, {p}{eng} (libzp {tab['lib_sha16']})",
           "",
           f"| stage | dispatches | us | GFLOP | TFLOP/s | {peak} | MFMA busy % | HBM MB (algorithmic) | HBM GB/s |",
           "|---|---|---|---|---|---|---|---|---|" + ("---|" if x3 else "")]
    for r in tab["stages"]:
        fr = f"{r['frac_of_peak']} | {r.get('frac_of_split_ceiling')}" if x3 else f"{r['frac_of_peak']}"
        out.append(f"| {r['stage']} | {r['dispatches']} | {r['us']} | {r['gflop']} | {r['tflops']} | {fr} "
                   f"| {r['mfma_busy_pct']} | {r['hbm_mb']} ({r['algo_mb']}) | {r['hbm_gbps']} |")
    return "\n".join(out) + "\n"


def write_leg_csv(tab, path):
    """One inference leg's last step, per kernel label (the dominant kernel's frac
    recomputable from one file): launches in the step, us per launch (kernel-trace pass), algorithmic
    TFLOP/s and its fraction of the leg's ceiling, HBM bytes per launch (PMC passes), MFMA busy %."""
    form = tab.get("split_form")
    ceil = PEAK_SPLIT[form] if form else PEAK[tab["precision"]]
    rows = sorted(tab["kernels"].items(), key=lambda kv: -kv[1]["launches"] * kv[1]["us_per_launch"])
    with open(path, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["label", "launches_per_step", "us_per_launch", "us_per_step", "tflops", "ceiling_tflops",
                    "frac_of_ceiling", "hbm_bytes_per_launch", "read_bytes_per_launch", "write_bytes_per_launch",
                    "mfma_busy_pct", "lib_sha16"])
        for k, v in rows:
            w.writerow([k, v["launches"], v["us_per_launch"], round(v["launches"] * v["us_per_launch"], 1), v["tflops"],
                        round(ceil, 1), round(v["tflops"] / ceil, 3) if v["tflops"] else None,
                        v["hbm_bytes_per_launch"], v["read_bytes_per_launch"], v["write_bytes_per_launch"],
                        v["mfma_busy_pct"], tab["lib_sha16"]])


def main(tag="r03", precs=("fp32", "bf16")):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    f = one(os.path.join(src, "stats", "**", "*kernel_stats.csv"))
    if f:
        shutil.copy(f, os.path.join(dst, f"{tag}_infer_kernel_stats.csv"))
    f = one(os.path.join(src, "train_1s", "**", "*kernel_stats.csv"))
    if f:
        shutil.copy(f, os.path.join(dst, f"{tag}_train1s_kernel_stats.csv"))
    traffic = {"source": f"tools/prof_r03.sh: rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate runs) over "
                         f"tools/prof_driver.py --mode infer --steps 3 --warmup 2, last step of each run",
               "correction": "bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 (FETCH_SIZE halves wide coalesced "
                             "reads on gfx950, MI355X_MICROARCH.md HBM section)",
               "by_label": {}, "kernels": {}}
    text = []
    for p in precs:
        tab = stage_table(src, p)
        traffic["lib_sha16"] = tab["lib_sha16"]
        for k, v in tab["kernels"].items():
            traffic["kernels"][k] = v
            if k.startswith("k_conv"):
                traffic["by_label"][k] = v["hbm_bytes_per_launch"]
        with open(os.path.join(dst, f"{tag}_stages_{p}.json"), "w") as fh:
            json.dump(tab, fh, indent=1)
        write_leg_csv(tab, os.path.join(dst, f"{tag}_{p}_step_kernels.csv"))
        with open(os.path.join(dst, f"{tag}_{p}_dispatches.csv"), "w", newline="") as fh:
            w = csv.writer(fh)
            keys = ["stage", "kernel", "geo", "us", "tflops", "read_mb", "write_mb", "algo_mb", "traffic_over_algo",
                    "mfma_busy_pct"]
            w.writerow(keys + ["lib_sha16"])
            for d in tab["dispatches"]:
                w.writerow([d[k] for k in keys] + [tab["lib_sha16"]])
        text.append(md(tab))
        print(md(tab))
    with open(os.path.join(dst, f"{tag}_pmc_traffic.json"), "w") as fh:
        json.dump(traffic, fh, indent=1)
    with open(os.path.join(dst, f"{tag}_stages.md"), "w") as fh:
        fh.write("\n".join(text))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0] if a else "r03", tuple(a[1:]) or ("fp32", "bf16"))
