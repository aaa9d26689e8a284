#!/bin/bash
# round 4, final tree: SQ counters + GRBM clock of the CG iteration's launch
# kinds (prologue, side, epilogue) at 200^4 -- one --pmc pass, kernel trace only
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r04_zl
mkdir -p $O
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $O/sq -o run --output-format csv -- python3 bench.py --steps 4 --warmup 2 --cpu-baseline off --lanczos 0 --grief off --matvec 0 > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections, json
rows = collections.defaultdict(dict)
meta = {}
for f in glob.glob("gpurun_out/r04_zl/sq/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mode_product" not in r["Kernel_Name"]:
            continue
        did = int(r["Dispatch_Id"])
        rows[did][r["Counter_Name"]] = float(r["Counter_Value"])
        meta[did] = (r["Kernel_Name"].split("(")[0],
                     (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
ids = sorted(rows)
last = ids[-8:]          # the last two CG iterations, 4 launches each
out = []
for k in range(4):
    dids = [last[k], last[4 + k]]
    m = {c: sum(rows[d].get(c, 0.0) for d in dids) / 2 for c in rows[dids[0]]}
    ms = sum(meta[d][1] for d in dids) / 2
    wc = m.get("SQ_WAVE_CYCLES", 1.0)
    rec = {"position": k, "kernel": meta[dids[0]][0], "ms": ms,
           "wait_any_frac": m.get("SQ_WAIT_ANY", 0) / wc,
           "wait_inst_any_frac": m.get("SQ_WAIT_INST_ANY", 0) / wc,
           "wait_inst_lds_frac": m.get("SQ_WAIT_INST_LDS", 0) / wc,
           "lds_bank_conflict": m.get("SQ_LDS_BANK_CONFLICT", 0),
           "clock_ghz": m.get("GRBM_GUI_ACTIVE", 0) / 8 / (ms * 1e-3) / 1e9 if ms else None,
           "mfma_busy_per_simd_frac": m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / 1024 /
               max(m.get("GRBM_GUI_ACTIVE", 1) / 8, 1),
           "per_launch": m}
    out.append(rec)
    print(json.dumps({k2: v for k2, v in rec.items() if k2 != "per_launch"}))
with open("gpurun_out/r04_zl/cg_sq.jsonl", "w") as f:
    for r in out:
        f.write(json.dumps(r) + "\n")
PY
echo done
