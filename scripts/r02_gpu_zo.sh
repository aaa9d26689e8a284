#!/bin/bash
# Round 2, session zo: prologue shape A/B repeated (GG_MP_PRO 0 / 1 interleaved).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02zo
mkdir -p $O
i=0
for v in 0 1 0 1 0 1; do
  i=$((i+1))
  GG_MP_PRO=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline off > $O/bench_$i.json 2> $O/bench_$i.err || { tail -5 $O/bench_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$i.json')); print('pro=$v', round(d['value'],3), round(d['ms_per_step'],2), [round(v,2) for v in d['mode_product_ms_by_position']])"
done
