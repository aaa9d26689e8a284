#!/bin/bash
# (run on the derived-r build; GG_CG_RDERIVE is not read by the main tree)
# round 4: CG prologue with r derived from the directions (GG_CG_RDERIVE=1,
# default) against the stored r (0): CG tests, then interleaved benches
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r04_zj
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fold.py tests/test_gpu_kron.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2 3; do
  for v in 1 0; do
    GG_CG_RDERIVE=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --grief off --lanczos 0 --matvec 0 > $O/b${v}_$i.json 2> $O/b${v}_$i.err || { tail -20 $O/b${v}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b${v}_$i.json'));print('rderive=$v', round(d['ms_per_step'],2), [round(v,2) for v in d['mode_product_ms_by_position']], round(d['closing_ms'],1), d['roofline']['traffic_source'][:40])"
  done
done
echo done
