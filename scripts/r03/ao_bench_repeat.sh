#!/bin/bash
# round 3, final tree: the default CG bench in 4 separate processes (the
# prologue launch level is drawn per process), Lanczos / GRIEF / CPU legs off
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03ao
mkdir -p $O
: > $O/rep.jsonl
for rep in 1 2 3 4; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --lanczos 0 --grief off > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print(json.dumps({'rep': $rep, 'value': d['value'], 'ms': d['ms_per_step'], 'pos': d['mode_product_ms_by_position'], 'traffic': d['roofline']['traffic']}))" >> $O/rep.jsonl
  tail -1 $O/rep.jsonl
done
