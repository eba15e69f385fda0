#!/usr/bin/env python3
"""Summarises a tools/prof_round.sh run (gpurun_out/prof_<tag>/) into profiles/:

  profiles/<tag>_infer_kernel_stats.csv   rocprofv3 --kernel-trace --stats, inference (bench.py)
  profiles/<tag>_train_kernel_stats.csv   same, training step (tools/prof_driver.py --mode train)
  profiles/<tag>_train_pmc_traffic.json   same two passes over training steps
  profiles/<tag>_pmc_traffic.json         HBM bytes per launch per kernel instantiation, from two
                                          separate --pmc passes (FETCH_SIZE, WRITE_SIZE) over eval
                                          inference steps, corrected as MI355X_MICROARCH.md §HBM
                                          prescribes: FETCH_SIZE and WRITE_SIZE are KiB; on gfx950
                                          FETCH_SIZE counts half the bytes of a wide coalesced read,
                                          so reads = 2 x FETCH_SIZE x 1024, writes = WRITE_SIZE x 1024.

bench.py reads the json's "by_label" map (keyed by its own kernel labels) for roofline.traffic.
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


def bench_label(name):
    """'void zp::k_conv<unsigned short, 4, 4, 4, 3, false>(zp_conv_args)' ->
    'k_conv<bf16,WC=4,WP=4,NWP=4,ST=3,smallC=0>' (the label bench.py / engine.py use)."""
    tn = {"unsigned short": "bf16", "_Float16": "f16", "float": "f32"}
    m = re.search(r"k_conv_strip<(unsigned short|_Float16), (\d+), (\d+), (\d+)>", name)
    if m:
        return f"k_conv_strip<{tn[m.group(1)]},WC={m.group(2)},ST={m.group(3)}>"
    m = re.search(r"k_conv_strip2<(unsigned short|_Float16), (\d+), (\d+), (true|false|\d+)(, (true|false))?(, (true|false))?>",
                  name)
    if m:  # (the 5th parameter, HEAD: the fused 16-bit head's conv, zp_conv2d_head; the 6th, BNR: a data
        # gradient taking the BN backward reduce -- same label, as the engine's)
        head = "_head" if m.group(6) == "true" else ""
        return f"k_conv_strip2{head}<{tn[m.group(1)]},WC={m.group(2)}>"
    sp = {"3": "x3", "2": "h2"}  # split-fp32 planes -> engine label
    m = re.search(r"k_conv3s<(\d+), (\d+)(?:, \d+)*>", name)
    if m:
        return f"k_conv3s<{sp[m.group(1)]},WC={m.group(2)}>"
    m = re.search(r"k_conv1x1n<(unsigned short|_Float16)(?:, \d+)?>", name)
    if m:  # the narrow-K 1x1 (round 5)
        return f"k_conv1x1n<{tn[m.group(1)]}>"
    if "k_stem_h2" in name:  # the direct two-plane stem (zp_stem_split)
        return "k_stem_h2"
    if re.search(r"k_conv3w32<(true|false)>", name):  # the 256 x 256 tile on 32x32x16 MFMAs (round 6, key 18)
        return "k_conv3w<h2>"  # (the engine's label: zp_conv2d_config reports the wide tile either way)
    # the 256 x 256 two-plane tile (+ fused head); template <ABL, DM, HEAD, SGB, PF, BF, STR, NUM, TPX>
    # (TPX 128: the 256 x 128 tile)
    m = re.search(r"k_conv3w<(\d+), (\d+), (true|false)((?:, (?:true|false|\d+))*)>", name)
    if m:
        rest = [v.strip() for v in m.group(4).split(",") if v.strip()]
        if m.group(3) == "true":
            return "k_conv3w_head<h2>"
        return "k_conv3w<h2,TP=128>" if len(rest) >= 6 and rest[5] == "128" else "k_conv3w<h2>"
    m = re.search(r"k_conv3<(\d+), (\d+), (\d+), (\d+), (\d+), (true|false)>", name)
    if m:
        return f"k_conv3<{sp[m.group(1)]},WC={m.group(2)},NWP={m.group(4)}>"
    m = re.search(r"k_conv_quad<(unsigned short|_Float16), (\d+), (true|false)>", name)
    if m:
        return f"k_conv_quad<{tn[m.group(1)]},W={m.group(2)}>"
    m = re.search(r"k_conv<(unsigned short|_Float16|float), (\d+), (\d+), (\d+), (\d+), (true|false)>", name)
    if not m:
        return None
    t = tn[m.group(1)]
    return (f"k_conv<{t},WC={m.group(2)},WP={m.group(3)},NWP={m.group(4)},ST={m.group(5)},"
            f"smallC={int(m.group(6) == 'true')}>")


def one(pattern):
    f = sorted(glob.glob(pattern, recursive=True))
    return f[0] if f else None


def counters(path, counter):
    per = defaultdict(list)
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if r["Counter_Name"] != counter:
                continue
            per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return per


def main(tag="r01"):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    for leg in ("infer", "train"):
        f = one(os.path.join(src, leg, "**", "*kernel_stats.csv"))
        if f:
            shutil.copy(f, os.path.join(dst, f"{tag}_{leg}_kernel_stats.csv"))
            print("copied", f)
    for pre, leg, what in (("pmc", "", "eval inference steps (--mode infer --steps 3 --warmup 1: R34 bs=32 bf16 "
                                         "eval + decode)"),
                           ("tpmc", "train_", "training steps (--mode train --steps 2 --warmup 1: R34 bs=32 bf16 "
                                              "forward + loss + backward + Adam)")):
        traffic(src, dst, tag, pre, leg, what)


def traffic(src, dst, tag, pre, leg, what):
    ff = one(os.path.join(src, f"{pre}_fetch", "**", "*counter_collection.csv"))
    fw = one(os.path.join(src, f"{pre}_write", "**", "*counter_collection.csv"))
    if not (ff and fw):
        print(f"no {pre} PMC passes found")
        return
    fetch, write = counters(ff, "FETCH_SIZE"), counters(fw, "WRITE_SIZE")
    out = {"source": f"tools/prof_round.sh: rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate runs) over "
                     f"tools/prof_driver.py {what}",
           "correction": "bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 (FETCH_SIZE halves wide coalesced "
                         "reads on gfx950, MI355X_MICROARCH.md HBM section)",
           "kernels": {}, "by_label": {}}
    for k in sorted(set(fetch) & set(write)):
        f, w = fetch[k], write[k]
        rd = 2.0 * 1024.0 * sum(f) / len(f)
        wr = 1024.0 * sum(w) / len(w)
        out["kernels"][k] = {"launches": len(f), "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                             "hbm_bytes_per_launch": rd + wr}
        lab = bench_label(k)
        if lab:
            out["by_label"][lab] = round(rd + wr)
    with open(os.path.join(dst, f"{tag}_{leg}pmc_traffic.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(f"== {tag}_{leg}pmc_traffic.json")
    for k, v in sorted(out["kernels"].items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * kv[1]["launches"])[:12]:
        print(f"{v['launches']:5d} {v['hbm_bytes_per_launch'] / 1e6:10.2f} MB/launch  {k[:100]}")

if __name__ == "__main__":
    main(*sys.argv[1:])
