#!/bin/bash
# round 3: split-K Gram, XCD-slab mapping (GG_GEMM_TN=14) vs default (3), slab counts
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03n
mkdir -p $O
: > $O/gram.jsonl
for sk in 8 16 24 32; do
for tn in 3 14; do
  GG_GEMM_TN=$tn GG_GEMM_SPLITK=$sk timeout -k 10 120 python -u tools/p2_kernels_bench.py --shapes 100000x1000,100000x5000 --what gram > $O/g.json 2> $O/g.err || { tail -5 $O/g.err; exit 1; }
  python -c "
import json
for l in open('$O/g.json'):
    d=json.loads(l); d.update(tn=$tn, splitk=$sk); print(json.dumps(d))" >> $O/gram.jsonl
done
done
cat $O/gram.jsonl
GG_GEMM_TN=14 GG_GEMM_SPLITK=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_grief.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest14.log 2>&1; rc=$?
tail -1 $O/pytest14.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest14.log | head -20; exit $rc; }
echo done
