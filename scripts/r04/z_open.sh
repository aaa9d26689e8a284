#!/bin/bash
# open-recurrence chain test + a short CG bench (closing after the timed region)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r04_z
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fold.py tests/test_gpu_kron.py tests/test_gpu_c3.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --grief off --lanczos 0 --matvec 0 > $O/b$i.json 2> $O/b$i.err || { tail -20 $O/b$i.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b$i.json'));print(round(d['value'],3), round(d['ms_per_step'],2), [round(v,2) for v in d['mode_product_ms_by_position']], 'closing', round(d['closing_ms'],2), d['roofline']['traffic_source'])"
done
