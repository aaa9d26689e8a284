"""Summarise a rocprofv3 kernel trace of one gg_potrf call (tuning aid).

Takes the last factorisation in the trace (from the launch after the last
torch copy / triangle kernel up to potrf_winv_kernel) and prints, per kernel
(and per grid height for the update kernel), the launch count, mean and total
duration, the factor's wall time and the wide-update GEMM rates.
Usage: python tools/potrf_trace.py <run_kernel_trace.csv> [panel columns]
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    pw = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    end = [i for i, r in enumerate(rows) if "potrf_winv" in r["Kernel_Name"]][-1]
    st = end
    while st > 0 and not ("triu" in rows[st]["Kernel_Name"] or "copyBuffer" in rows[st]["Kernel_Name"]):
        st -= 1
    seg = rows[st + 1:end + 1]
    t0 = int(seg[0]["Start_Timestamp"])
    agg = collections.defaultdict(list)
    for r in seg:
        name = r["Kernel_Name"].split("(")[0][-30:]
        key = (name, r["Grid_Size_Y"] if "upd" in name else "", r["Stream_Id"])
        agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    print("factor wall us %.1f" % ((int(seg[-1]["End_Timestamp"]) - t0) / 1000.0))
    for k, v in sorted(agg.items()):
        print("  %-32s y=%-4s q%s  n=%-4d mean %7.1f us  sum %8.1f us" % (k[0], k[1], k[2], len(v),
                                                                     sum(v) / len(v), sum(v)))
    tf = []
    for r in seg:
        if "gemm_tn" in r["Kernel_Name"]:
            M = int(r["Grid_Size_X"]) // 256 * 128
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
            tf.append("%d:%.0f" % (M, M * M * pw / (d * 1e-6) / 1e12))
    print("  wide-update TF by M:", " ".join(tf[:16]))


if __name__ == "__main__":
    main()
