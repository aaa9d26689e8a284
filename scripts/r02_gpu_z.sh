#!/bin/bash
# Round 2, session z: persistent XCD-grouped TN Gram (variants 6, 7) vs the
# launch-order kernel (3): GEMM tests, timings, L2 hit counters.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02z
mkdir -p $O
for v in 6 7 3; do
  GG_GEMM_TN=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_grief.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or cholesky or fixtures_model" > $O/pytest_tn$v.log 2>&1 || { echo "variant $v FAILED"; grep -E "^E |FAILED" $O/pytest_tn$v.log | head; exit 1; }
  echo "variant $v tests: $(tail -1 $O/pytest_tn$v.log)"
  GG_GEMM_TN=$v timeout -k 10 300 python -u tools/p2_kernels_bench.py --what gram > $O/gram_tn$v.jsonl 2>> $O/gram.err || exit $?
  python -c "import json;[print('variant $v', json.loads(l)['p'], round(json.loads(l)['ms'],2), round(json.loads(l)['tflops'],1)) for l in open('$O/gram_tn$v.jsonl')]"
done
G="python -u tools/p2_kernels_bench.py --what gram --shapes 100000x10000"
GG_GEMM_TN=6 timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --kernel-trace -d $O/gram_tcc6 -o run --output-format csv -- $G > $O/gram_tcc6.log 2>&1 || { tail -5 $O/gram_tcc6.log; exit 1; }
python - <<'PY'
import csv
from collections import defaultdict
agg=defaultdict(float); ids=set()
for r in csv.DictReader(open("gpurun_out/r02z/gram_tcc6/run_counter_collection.csv")):
    if "gemm_tn" not in r["Kernel_Name"]: continue
    agg[r["Counter_Name"]]+=float(r["Counter_Value"]); ids.add(r["Dispatch_Id"])
n=len(ids); print({k: round(v/n/1e6,1) for k,v in agg.items()})
PY
