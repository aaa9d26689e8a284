"""HBM traffic per launch of the fused-CG mode products from rocprofv3 PMC passes.

usage: python tools/pmc_traffic.py RD_DIR WR_DIR OUT_JSON [--fusion F] [--xdefer MODE] [--rq 0|1]

Counters (two separate --pmc runs of `bench.py --steps 2 --warmup 1`, kernel
trace only, as MI355X_MICROARCH.md prescribes):
  reads   TCC_EA0_RDREQ_32B_sum, _64B_sum, _128B_sum (L2 -> fabric requests by size)
  writes  TCC_EA0_WRREQ_sum, TCC_EA0_WRREQ_64B_sum
bytes = 32 N32 + 64 N64 + 128 N128 (reads), 64 N64 (writes) -- the request
sizes themselves, not FETCH_SIZE (which tallies 128-B requests at 64 B on
gfx950).  Calibration on the kernel's own access pattern: the plain mode
product (launch position 2) reads X exactly once (12.8 GB at 200^4) and
writes Y once, so its counted bytes must equal those; the result records the
ratio.  The dominant launch (position 0, CG prologue) is read from the
iterations whose fused update was pending (the third CG iteration onwards).
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
            if "mode_product" not in r["Kernel_Name"]:
                continue
            did = int(r["Dispatch_Id"])
            out[did][r["Counter_Name"]] = float(r["Counter_Value"])
            names[did] = r["Kernel_Name"].split("(")[0]
    return out, names


def main():
    rd_dir, wr_dir, out = sys.argv[1:4]
    fusion = int(sys.argv[sys.argv.index("--fusion") + 1]) if "--fusion" in sys.argv else 0
    # the x-update schedule the passes were taken with (gg_cg_set_xdefer mode;
    # the library default 2 unless GG_CG_XDEFER overrides it)
    xdefer = (int(sys.argv[sys.argv.index("--xdefer") + 1]) if "--xdefer" in sys.argv
              else int(os.environ.get("GG_CG_XDEFER", "2")))
    # the r.q source (gg_cg_set_rq; the library default 1 unless GG_CG_RQ=0)
    rq = (int(sys.argv[sys.argv.index("--rq") + 1]) if "--rq" in sys.argv
          else int(os.environ.get("GG_CG_RQ", "1") != "0"))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    rd, names = dispatches(rd_dir)
    wr, _ = dispatches(wr_dir)
    ids = sorted(rd)
    d = 4
    iters = [ids[i:i + d] for i in range(0, len(ids) - d + 1, d)]
    # the last two iterations: fully fused (pending updates), and with the
    # deferred x update one with and one without the x pass -- averaged, as
    # bench.launch_passes counts them
    last2 = iters[-2:]
    per_pos = []
    for k in range(d):
        dids = [it[k] for it in last2]
        rbytes = sum(sum(rd[did].get(c, 0.0) * s for c, s in SIZES.items())
                     for did in dids) / len(dids)
        wbytes = sum(wr.get(did, {}).get("TCC_EA0_WRREQ_64B_sum", 0.0) * 64
                     for did in dids) / len(dids)
        per_pos.append({"position": k, "kernel": names[dids[-1]], "read_bytes": rbytes,
                        "write_bytes": wbytes, "traffic_bytes": rbytes + wbytes,
                        "dispatches": dids})
    n = 200 ** 4
    passes = [float(v) for v in bench.launch_passes(d, "fused", fusion, xdefer, rq and not fusion)]
    for k, pp in enumerate(per_pos):
        pp["algorithmic_bytes"] = passes[k] * 8.0 * n
        pp["ratio"] = pp["traffic_bytes"] / pp["algorithmic_bytes"]
    tot = sum(pp["traffic_bytes"] for pp in per_pos)
    calib = {"iteration_ratio": tot / (sum(passes) * 8.0 * n),
             "per_position_ratio": [pp["ratio"] for pp in per_pos]}
    dom = per_pos[0]
    fold_mask = sum(1 << k for k, pp in enumerate(per_pos) if "fold" in pp["kernel"])
    res = {
        "position": 0, "recurrence": "fused", "fusion_layout": fusion, "x_deferred": xdefer,
        "rq_identity": int(bool(rq and not fusion)),
        "fold_mask": fold_mask,
        # bench.py reuses these counters only for kernels built from the same sources
        "source_sha256": bench.kernel_source_hash(),
        "sources": bench.KERNEL_SOURCES,
        "kernel": dom["kernel"], "traffic_bytes": dom["traffic_bytes"],
        "read_bytes": dom["read_bytes"], "write_bytes": dom["write_bytes"],
        "algorithmic_bytes": passes[0] * 8.0 * n,
        "calibrated_on_own_pattern": all(abs(pp["ratio"] - 1) < 0.05 for pp in per_pos),
        "calibration": calib, "per_position": per_pos,
        "method": "separate rocprofv3 --pmc passes (reads by request size / writes), kernel "
                  "trace only, bench.py --steps 4 --warmup 2 at 200^4; bytes = request "
                  "counts x request sizes, averaged over the last two iterations; checked "
                  "per launch against its algorithmic passes (%s x 12.8 GB) on the "
                  "kernels' own patterns" % " / ".join("%g" % v for v in passes),
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "per_position"}))


if __name__ == "__main__":
    main()
