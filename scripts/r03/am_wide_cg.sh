#!/bin/bash
# round 3: 12-wave workgroups in the fused CG (GG_FOLD_PRO_W=12 prologue,
# GG_FOLD_SIDE_W=12 side launches): CG parity with both on, then interleaved
# bench processes
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03am
mkdir -p $O
GG_FOLD_PRO_W=12 GG_FOLD_SIDE_W=12 timeout -k 10 400 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_kron.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_wide.log 2>&1 || { grep -E "^E |FAILED" $O/pytest_wide.log | head -20; tail -3 $O/pytest_wide.log; exit 1; }
tail -1 $O/pytest_wide.log
B="python -u bench.py --steps 10 --warmup 3 --cpu-baseline off --lanczos 0 --grief off"
: > $O/ab.jsonl
for rep in 1 2; do
for v in "0 0" "12 0" "0 12" "12 12"; do
  set -- $v
  GG_FOLD_PRO_W=$1 GG_FOLD_SIDE_W=$2 timeout -k 10 200 $B > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print(json.dumps({'pro_w': $1, 'side_w': $2, 'ms': d['ms_per_step'], 'pos': d['mode_product_ms_by_position']}))" >> $O/ab.jsonl
  tail -1 $O/ab.jsonl
done
done
