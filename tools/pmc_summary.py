"""Summarise rocprofv3 --pmc counter_collection.csv files per kernel.

usage: python tools/pmc_summary.py DIR [DIR ...]
Prints, per kernel name (shortened) and counter, the per-dispatch mean and
the mean duration.  FETCH_SIZE / WRITE_SIZE are in KB (rocprofv3 units).
"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name)
    return name[:90]


def main(dirs):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                dur[k][(f, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) -
                                                 int(r["Start_Timestamp"])) * 1e-6
    for k in sorted(agg, key=lambda k: -sum(dur[k].values())):
        ds = list(dur[k].values())
        print("%s  dispatches=%d mean_ms=%.3f" % (k, len(ds) // max(1, len(dirs)) or len(ds),
                                                  sum(ds) / len(ds)))
        for c, v in sorted(agg[k].items()):
            print("    %-26s mean %.6g" % (c, sum(v) / len(v)))


if __name__ == "__main__":
    main(sys.argv[1:])
