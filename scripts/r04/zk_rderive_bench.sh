#!/bin/bash
# (run on the derived-r build; GG_CG_RDERIVE is not read by the main tree)
# round 4: interleaved 200^4 CG benches, r derived (1) vs stored (0)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r04_zk
mkdir -p $O
for i in 1 2; do
  for v in 1 0; do
    GG_CG_RDERIVE=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --grief off --lanczos 0 --matvec 0 > $O/b${v}_$i.json 2> $O/b${v}_$i.err || { tail -20 $O/b${v}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b${v}_$i.json'));print('rderive=$v', round(d['ms_per_step'],2), [round(v,2) for v in d['mode_product_ms_by_position']], round(d['closing_ms'],1))"
  done
done
echo done
