#!/bin/bash
# round 4: C2 Gram (n = 1e5, p = 1000) split-K slab count: 36 lower tiles x
# slabs per XCD onto 96 slots (16 slabs: one 75 % round; 64: three full rounds)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r04zh
mkdir -p $O
: > $O/ab.jsonl
for rep in 1 2; do
 for s in 16 64 40 32 48 80; do
  GG_GEMM_SPLITK=$s timeout -k 10 200 python -u tools/p2_kernels_bench.py --shapes 100000x1000,100000x2000 --what gram > $O/t.jsonl 2> $O/t.err || { tail -5 $O/t.err; exit 1; }
  python -c "
import json
for l in open('$O/t.jsonl'):
    d=json.loads(l); d['splitk']=$s; d['rep']=$rep; print(json.dumps(d))" >> $O/ab.jsonl
  tail -2 $O/ab.jsonl
 done
done
echo done
