#!/bin/bash
# round 3: Cholesky wide-update GEMM variant (GG_GEMM_TN) x panel width
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03t
mkdir -p $O
: > $O/ab.jsonl
for tn in 14 6 7 10 2; do
 for pw in 256 512; do
  GG_GEMM_TN=$tn GG_POTRF_PANEL=$pw timeout -k 10 300 python -u tools/p2_kernels_bench.py --shapes 20000x5000,20000x10000 --what potrf > $O/t.jsonl 2> $O/t.err || { tail -5 $O/t.err; exit 1; }
  python -c "
import json
for l in open('$O/t.jsonl'):
    d=json.loads(l); d['panel']=$pw; d['tn']=$tn; print(json.dumps(d))" >> $O/ab.jsonl
 done
done
cat $O/ab.jsonl
echo done
