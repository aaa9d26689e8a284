#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r04_za
mkdir -p $O
for i in 1 2; do
  for f in 0 1; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --grief off --lanczos 0 --matvec 0 --fusion $f > $O/b${f}_$i.json 2> $O/b${f}_$i.err || { tail -20 $O/b${f}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b${f}_$i.json'));print('fusion=$f', round(d['ms_per_step'],2), [round(v,2) for v in d['mode_product_ms_by_position']])"
  done
done
