#!/bin/bash
# SQ counters + GRBM clock of the plain folded mode product: chunked kernel
# (GG_FOLD_RING=0) vs ring variants 1 and 5 -- one --pmc pass each, kernel
# trace only; plus the available-counter list for later passes.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r04_c
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
for v in 0 1 5; do
  GG_FOLD_RING=$v timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d $O/v$v -o run --output-format csv -- python3 tools/matvec_bench.py --reps 2 > $O/v$v.log 2>&1 || { tail -5 $O/v$v.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, json
for v in ("0", "1", "5"):
    agg = collections.defaultdict(list)
    dur = []
    for f in glob.glob("gpurun_out/r04_c/v%s/**/*counter_collection.csv" % v, recursive=True):
        seen = set()
        for r in csv.DictReader(open(f)):
            if "mode_product" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
                k = r["Dispatch_Id"]
                if k not in seen:
                    seen.add(k)
                    dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    m = {k: sum(x) / len(x) for k, x in agg.items()}
    wc = m.get("SQ_WAVE_CYCLES", 1.0)
    ms = sum(dur) / max(len(dur), 1)
    out = {"variant": v, "ms": ms, "per_launch": m,
           "wait_any_frac": m.get("SQ_WAIT_ANY", 0) / wc,
           "wait_inst_any_frac": m.get("SQ_WAIT_INST_ANY", 0) / wc,
           "clock_ghz": m.get("GRBM_GUI_ACTIVE", 0) / 8 / (ms * 1e-3) / 1e9 if ms else None,
           "mfma_busy_per_simd_frac": m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / 1024 /
               (m.get("GRBM_GUI_ACTIVE", 1) / 8)}
    print(json.dumps(out))
    open("gpurun_out/r04_c/summary.jsonl", "a").write(json.dumps(out) + "\n")
PY
