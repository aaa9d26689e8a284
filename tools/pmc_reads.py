"""Reads per block-CG launch from one rocprofv3 --pmc pass of the RDREQ
counters (diag companion of tools/pmc_block.py).  usage: pmc_reads.py DIR"""
import csv
import glob
import os
import sys
from collections import defaultdict

SIZES = {"TCC_EA0_RDREQ_32B_sum": 32, "TCC_EA0_RDREQ_64B_sum": 64,
         "TCC_EA0_RDREQ_128B_sum": 128}
rd, names = defaultdict(float), {}
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "blk_mode" in k or "blk_pair" in k:
            did = int(r["Dispatch_Id"])
            rd[did] += float(r["Counter_Value"]) * SIZES.get(r["Counter_Name"], 0)
            names[did] = k.split("(")[0]
ids = sorted(rd)[-6:]
for did in ids:
    print("%-48s rd %.2f GB" % (names[did][:48], rd[did] / 1e9))
