"""Summarise one rocprofv3 --pmc pass (SQ_* / GRBM_* counters) of the mode
products: per-launch means, wave-wait fractions, clock and MFMA busy per SIMD.

usage: python tools/sq_summary.py DIR LABEL [KERNEL_SUBSTRING]"""
import collections
import csv
import glob
import json
import os
import sys


def main(d, label, sub="mode_product"):
    agg = collections.defaultdict(list)
    dur = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
                dur[(f, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) -
                                              int(r["Start_Timestamp"])) * 1e-6
    m = {k: sum(x) / len(x) for k, x in agg.items()}
    ms = sum(dur.values()) / max(len(dur), 1)
    wc = m.get("SQ_WAVE_CYCLES", 1.0)
    gui = m.get("GRBM_GUI_ACTIVE", 0.0)
    out = {"label": label, "ms": ms, "per_launch": m,
           "wait_any_frac": m.get("SQ_WAIT_ANY", 0) / wc,
           "wait_inst_any_frac": m.get("SQ_WAIT_INST_ANY", 0) / wc,
           "clock_ghz": gui / 8 / (ms * 1e-3) / 1e9 if ms and gui else None,
           "mfma_busy_per_simd_frac": (m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / 1024 / (gui / 8)
                                       if gui else None)}
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:])
