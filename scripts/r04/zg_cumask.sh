#!/bin/bash
# round 4: Cholesky wide update on a CU-masked stream (GG_POTRF_CUMASK=R
# leaves R CUs of every 32 to the chain) against the low-priority stream
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r04zg
mkdir -p $O
: > $O/ab.jsonl
for rep in 1 2; do
 for r in 0 4 8 2 12; do
  if [ $r = 0 ]; then unset GG_POTRF_CUMASK; else export GG_POTRF_CUMASK=$r; fi
  timeout -k 10 200 python -u tools/p2_kernels_bench.py --shapes 20000x10000,12000x5000 --what potrf > $O/t.jsonl 2> $O/t.err || { tail -5 $O/t.err; exit 1; }
  python -c "
import json
for l in open('$O/t.jsonl'):
    d=json.loads(l); d['cumask']=$r; d['rep']=$rep; print(json.dumps(d))" >> $O/ab.jsonl
  tail -2 $O/ab.jsonl
 done
done
echo done
