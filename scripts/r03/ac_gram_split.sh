#!/bin/bash
# round 3: small-p Gram split-K factor A/B on the XCD-slab grid (C2: n = 1e5, p = 1000; p = 2000)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03ac
mkdir -p $O
: > $O/gram.jsonl
for S in 16 24 32 40 48 64 96; do
  GG_GEMM_SPLITK=$S timeout -k 10 200 python -u tools/p2_kernels_bench.py --shapes 100000x1000,100000x2000 --what gram > $O/g.json 2> $O/g.err || { tail -5 $O/g.err; exit 1; }
  python -c "
import json
for l in open('$O/g.json'):
    d=json.loads(l); d.update(S=$S); print(json.dumps(d))" >> $O/gram.jsonl
done
cat $O/gram.jsonl
echo done
