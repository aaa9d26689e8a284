#!/bin/bash
# round 3: kLean A addressing in the fused CG (GG_FOLD_LEAN for the side /
# epilogue launches, GG_FOLD_LEAN_PRO=1/2 for the prologue): parity tests
# with the knobs on, then interleaved bench processes (the prologue launch
# level is drawn per process)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03ak
mkdir -p $O
GG_FOLD_LEAN=1 GG_FOLD_LEAN_PRO=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_kron.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_lean2.log 2>&1 || { grep -E "^E |FAILED" $O/pytest_lean2.log | head -20; tail -3 $O/pytest_lean2.log; exit 1; }
tail -1 $O/pytest_lean2.log
B="python -u bench.py --steps 10 --warmup 3 --cpu-baseline off --lanczos 0 --grief off"
: > $O/ab.jsonl
for rep in 1 2; do
for v in "0 0" "1 0" "1 1" "1 2"; do
  set -- $v
  GG_FOLD_LEAN=$1 GG_FOLD_LEAN_PRO=$2 timeout -k 10 200 $B > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print(json.dumps({'lean': $1, 'lean_pro': $2, 'ms': d['ms_per_step'], 'pos': d['mode_product_ms_by_position']}))" >> $O/ab.jsonl
  tail -1 $O/ab.jsonl
done
done
