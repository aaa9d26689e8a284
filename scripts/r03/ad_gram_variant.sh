#!/bin/bash
# round 3: small-p Gram, TN kernel variant A/B (GG_GEMM_TN) at C2 shapes
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03ad
mkdir -p $O
: > $O/gram.jsonl
for tn in 14 3 1 2 11 12 13 6 8; do
  GG_GEMM_TN=$tn timeout -k 10 200 python -u tools/p2_kernels_bench.py --shapes 100000x1000,100000x2000 --what gram > $O/g.json 2> $O/g.err || { tail -5 $O/g.err; exit 1; }
  python -c "
import json
for l in open('$O/g.json'):
    d=json.loads(l); d.update(tn=$tn); print(json.dumps(d))" >> $O/gram.jsonl
done
cat $O/gram.jsonl
echo done
