#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc SQ passes over tools/conv3_ab.py (round 6, tools/plans/r06_g9.txt):
per kernel (the conv launches of the layer under test), counters averaged over its dispatches.

  SQ_WAVE_CYCLES = SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY (MI355X_MICROARCH.md: disjoint;
  quad-cycles): the share of wave lifetime parked on s_waitcnt / s_barrier, stalled at issue
  (dependency / pipe busy; SQ_WAIT_INST_LDS its LDS-issue part), and issuing.
  MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024) (tools/prof_stages.py).
  LDS: SQ_LDS_BANK_CONFLICT extra cycles over SQ_LDS_IDX_ACTIVE array cycles.
usage: python tools/sq_summary.py gpurun_out/g9 [> profiles/r06_sq_counters.md]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    per = defaultdict(lambda: defaultdict(float))
    n = defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "zp::k_conv" not in k:
                continue
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[k].add(r["Dispatch_Id"])
    return {k: {c: v / len(n[k]) for c, v in cs.items()} for k, cs in per.items()}, {k: len(v) for k, v in n.items()}


def main(root):
    print("| layer | kernel | dispatches | wait (s_waitcnt / barrier) | issue stall | of which LDS issue | issuing | MFMA busy | LDS bank-conflict cycles / array cycles | LDS / VALU / SALU / VMEM instr per wave |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for lay in sorted({os.path.basename(p).split("_", 1)[1] for p in glob.glob(os.path.join(root, "sq*_*"))}):
        a, na = load(os.path.join(root, f"sqA_{lay}"))
        b, nb = load(os.path.join(root, f"sqB_{lay}"))
        for k in sorted(set(a) & set(b)):
            A, B = a[k], b[k]
            wc = A.get("SQ_WAVE_CYCLES", 0.0) or 1.0
            waves = A.get("SQ_WAVES", 0.0) or 1.0
            grbm = B.get("GRBM_GUI_ACTIVE", 0.0)
            busy = 100.0 * B.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (grbm / 8.0 * 1024.0) if grbm else float("nan")
            lds = B.get("SQ_LDS_IDX_ACTIVE", 0.0)
            short = k.split("(")[0].replace("void zp::", "")[:60]
            print(f"| {lay} | {short} | {na[k]} | {100 * A.get('SQ_WAIT_ANY', 0) / wc:.1f}% | "
                  f"{100 * A.get('SQ_WAIT_INST_ANY', 0) / wc:.1f}% | {100 * A.get('SQ_WAIT_INST_LDS', 0) / wc:.1f}% | "
                  f"{100 * A.get('SQ_ACTIVE_INST_ANY', 0) / wc:.1f}% | {busy:.1f}% | "
                  f"{A.get('SQ_LDS_BANK_CONFLICT', 0):.3g} / {lds:.3g} | "
                  f"{B.get('SQ_INSTS_LDS', 0) / waves:.0f} / {B.get('SQ_INSTS_VALU', 0) / waves:.0f} / "
                  f"{B.get('SQ_INSTS_SALU', 0) / waves:.0f} / {B.get('SQ_INSTS_VMEM', 0) / waves:.0f} |")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/g9")
