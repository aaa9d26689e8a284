#!/bin/bash
# round 3: SQ counters of the plain folded mode product (4-wave kLean default
# vs 12-wave workgroups, GG_FOLD_VARIANT=15) -- one --pmc pass each, kernel
# trace only
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03ap
mkdir -p $O
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
for v in 0 15; do
  GG_FOLD_VARIANT=$v timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d $O/v$v -o run --output-format csv -- python3 tools/matvec_bench.py --reps 2 > $O/v$v.log 2>&1 || { tail -5 $O/v$v.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, json
for v in ("0", "15"):
    agg = collections.defaultdict(list)
    for f in glob.glob("gpurun_out/r03ap/v%s/**/*counter_collection.csv" % v, recursive=True):
        for r in csv.DictReader(open(f)):
            if "mode_product" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(x) / len(x) for k, x in agg.items()}
    wc = m.get("SQ_WAVE_CYCLES", 1.0)
    out = {"variant": v, "per_launch": m,
           "wait_any_frac": m.get("SQ_WAIT_ANY", 0) / wc,
           "wait_inst_any_frac": m.get("SQ_WAIT_INST_ANY", 0) / wc,
           "mfma_busy_over_busy": m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(m.get("SQ_BUSY_CYCLES", 1), 1)}
    print(json.dumps(out))
    open("gpurun_out/r03ap/summary.jsonl", "a").write(json.dumps(out) + "\n")
PY
