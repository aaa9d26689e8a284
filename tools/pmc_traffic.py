"""HBM traffic per launch of the dominant kernel from rocprofv3 PMC passes.

usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR CALIB_FETCH_DIR KERNEL_SUBSTR OUT_JSON

FETCH_SIZE is calibrated for the mode product's A-operand access shape by
tools/fetch_calib (kernel `kfrag`: 8 B per lane, 4 rows x 128 B per wave
instruction): bytes = FETCH_SIZE[KB] * 1024 * (true bytes / counted bytes of
kfrag).  WRITE_SIZE is taken as bytes (MI355X_MICROARCH.md: exact for
streaming stores).  Counters were collected in separate passes with
--kernel-trace only, as the guide prescribes.
"""
import csv
import glob
import json
import os
import sys


def rows(d):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def mean_counter(d, sub, counter):
    v = [float(r["Counter_Value"]) for r in rows(d)
         if sub in r["Kernel_Name"] and r["Counter_Name"] == counter]
    names = {r["Kernel_Name"].split("(")[0] for r in rows(d) if sub in r["Kernel_Name"]}
    return sum(v) / len(v), len(v), sorted(names)


def main():
    fdir, wdir, cdir, sub, out = sys.argv[1:6]
    calib_bytes = 2147483200.0  # tools/fetch_calib kfrag: R * M * 8
    kf, _, _ = mean_counter(cdir, "kfrag", "FETCH_SIZE")
    factor = calib_bytes / (kf * 1024.0)
    fetch, n, names = mean_counter(fdir, sub, "FETCH_SIZE")
    write, _, _ = mean_counter(wdir, sub, "WRITE_SIZE")
    res = {
        "kernel": names[0] if len(names) == 1 else names,
        "dispatches": n,
        "fetch_size_kb": fetch,
        "write_size_kb": write,
        "fetch_calibration": factor,
        "read_bytes": fetch * 1024.0 * factor,
        "write_bytes": write * 1024.0,
        "traffic_bytes": fetch * 1024.0 * factor + write * 1024.0,
        "method": "separate --pmc FETCH_SIZE / WRITE_SIZE passes (kernel trace only); "
                  "FETCH_SIZE scaled by the kfrag calibration of tools/fetch_calib",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
