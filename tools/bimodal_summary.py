"""Per-process, per-launch-position TCC read latency and DRAM credit stalls of
the fused-CG mode products (scripts/r04/k_bimodal.sh output): the first
(prologue) launch's level against the others'."""
import collections
import csv
import glob
import os
import sys


def main(root):
    for d in sorted(glob.glob(os.path.join(root, "p*"))):
        if not os.path.isdir(d):
            continue
        rows = collections.defaultdict(dict)
        meta = {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "mode_product" not in r["Kernel_Name"]:
                    continue
                k = int(r["Dispatch_Id"])
                rows[k][r["Counter_Name"]] = float(r["Counter_Value"])
                meta[k] = ((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6,
                           r["Kernel_Name"][:60])
        ks = sorted(rows)
        # fused CG, d = 4: launches come in fours (prologue, side, side, epilogue)
        by_pos = collections.defaultdict(list)
        for i, k in enumerate(ks):
            by_pos[i % 4].append((meta[k][0], rows[k]))
        print(os.path.basename(d))
        for pos in range(4):
            v = by_pos[pos][2:]   # skip the warm-up iterations
            if not v:
                continue
            ms = sum(t for t, _ in v) / len(v)
            rd = sum(c.get("TCC_EA0_RDREQ_sum", 0) for _, c in v)
            lv = sum(c.get("TCC_EA0_RDREQ_LEVEL_sum", 0) for _, c in v)
            st = sum(c.get("TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum", 0) for _, c in v) / len(v)
            wr = sum(c.get("TCC_EA0_WRREQ_sum", 0) for _, c in v) / len(v)
            print("  pos %d  %.3f ms  rd_latency %.0f cyc  dram_credit_stall %.3g  rdreq %.4g  wrreq %.4g"
                  % (pos, ms, lv / rd if rd else 0, st, rd / len(v), wr))


if __name__ == "__main__":
    main(sys.argv[1])
