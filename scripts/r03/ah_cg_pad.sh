#!/bin/bash
# round 3: stagger of the CG vectors inside the work buffer (GG_CG_PAD elements): interleaved A/B of the 200^4 iteration
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03ah
mkdir -p $O
: > $O/ab.jsonl
for rep in 1 2; do
 for pad in 0 32 512 2080 8224; do
  GG_CG_PAD=$pad timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline off --lanczos 0 --grief off > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python -c "
import json
d=json.load(open('$O/b.json')); print(json.dumps({'pad': $pad, 'rep': $rep, 'value': d['value'], 'ms': d['ms_per_step'], 'pos': [round(v,2) for v in d['mode_product_ms_by_position']]}))" >> $O/ab.jsonl
 done
done
cat $O/ab.jsonl
echo done
