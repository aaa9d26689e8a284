"""HBM traffic per launch of the block-basis fused CG (gg_kronb.hip) from two
rocprofv3 PMC passes, as tools/pmc_traffic.py does for the grid basis.

usage: python tools/pmc_block.py RD_DIR WR_DIR OUT_JSON [XWIN [RDERIVE]]

XWIN: the x window the runs took (gg_cg_get_xwin; default GG_CG_XWIN or the
library default 8; 0 = mode 2's balanced pairs).

Counters (separate --pmc runs of `bench.py --steps 2 --warmup 10 --matvec 0
--lanczos 0 --grief off --cpu-baseline off` -- 12 iterations, so the last two
carry the full x window; PMC_BENCH_STEPS overrides the label --, kernel trace only, per
MI355X_MICROARCH.md): reads TCC_EA0_RDREQ_{32B,64B,128B}_sum, writes
TCC_EA0_WRREQ_64B_sum; bytes = request counts x request sizes.  The launches
of one iteration are the three blk_* kernels (prologue, plain mode product,
pair + epilogue + x side job); the last two iterations are averaged and each
launch is checked against its algorithmic passes (bench.block_launch_passes).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIZES = {"TCC_EA0_RDREQ_32B_sum": 32, "TCC_EA0_RDREQ_64B_sum": 64,
         "TCC_EA0_RDREQ_128B_sum": 128}


def dispatches(d):
    out = defaultdict(dict)
    names = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "blk_mode" not in r["Kernel_Name"] and "blk_pair" not in r["Kernel_Name"]:
                continue
            did = int(r["Dispatch_Id"])
            out[did][r["Counter_Name"]] = float(r["Counter_Value"])
            names[did] = r["Kernel_Name"].split("(")[0]
    return out, names


def main():
    rd_dir, wr_dir, out = sys.argv[1:4]
    xwin = int(sys.argv[4]) if len(sys.argv) > 4 else int(os.environ.get("GG_CG_XWIN", "8"))
    xwin = xwin if xwin >= 2 else 0
    rder = bool(int(sys.argv[5])) if len(sys.argv) > 5 else \
        (xwin >= 2 and os.environ.get("GG_CG_RDERIVE", "1") != "0")
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    rd, names = dispatches(rd_dir)
    wr, _ = dispatches(wr_dir)
    ids = sorted(rd)
    d, L = 4, 3
    iters = [ids[i:i + L] for i in range(0, len(ids) - L + 1, L)]
    last2 = iters[-2:]
    n = 200 ** 4
    passes = [float(v) for v in bench.block_launch_passes(d, xwin, rder)]
    per_pos = []
    for k in range(L):
        dids = [it[k] for it in last2]
        rbytes = sum(sum(rd[did].get(c, 0.0) * s for c, s in SIZES.items())
                     for did in dids) / len(dids)
        wbytes = sum(wr.get(did, {}).get("TCC_EA0_WRREQ_64B_sum", 0.0) * 64
                     for did in dids) / len(dids)
        pp = {"position": k, "kernel": names[dids[-1]], "read_bytes": rbytes,
              "write_bytes": wbytes, "traffic_bytes": rbytes + wbytes, "dispatches": dids,
              "algorithmic_bytes": passes[k] * 8.0 * n}
        pp["ratio"] = pp["traffic_bytes"] / pp["algorithmic_bytes"]
        per_pos.append(pp)
    tot = sum(pp["traffic_bytes"] for pp in per_pos)
    res = {
        "block_basis": True, "recurrence": "fused", "fusion_layout": 0, "x_deferred": 2, "x_window": xwin, "r_derived": rder,
        "rq_identity": 1, "fold_mask": 0,
        "source_sha256": bench.kernel_source_hash(),
        "sources": bench.KERNEL_SOURCES,
        "calibrated_on_own_pattern": all(abs(pp["ratio"] - 1) < 0.05 for pp in per_pos),
        "calibration": {"iteration_ratio": tot / (sum(passes) * 8.0 * n),
                        "per_position_ratio": [pp["ratio"] for pp in per_pos]},
        "per_position": per_pos,
        "method": "separate rocprofv3 --pmc passes (reads by request size / writes), kernel "
                  "trace only, bench.py %s at 200^4 (block basis); bytes = "
                  "request counts x request sizes, averaged over the last two iterations; "
                  "checked per launch against its algorithmic passes (%s x 12.8 GB)"
                  % (os.environ.get("PMC_BENCH_STEPS", "--steps 2 --warmup 10"),
                     " / ".join("%g" % v for v in passes)),
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "per_position"}))


if __name__ == "__main__":
    main()
