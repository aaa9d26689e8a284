#!/bin/bash
# Round 2, session zn: fused-CG prologue launch shape A/B (GG_MP_PRO 0..3) at
# 200^4: bench iterations, per-position launch times; C3 CG residual test on each.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02zn
mkdir -p $O
for v in 0 1 2 3 0; do
  GG_MP_PRO=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline off > $O/bench_pro$v.json 2> $O/bench_pro$v.err || { tail -5 $O/bench_pro$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_pro$v.json')); print('pro=$v', round(d['value'],3), round(d['ms_per_step'],2), [round(v,2) for v in d['mode_product_ms_by_position']])"
done
for v in 1 2 3; do
  GG_MP_PRO=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_c3.py -m gpu -x -q --timeout 200 --timeout-method thread -k "cg_true" > $O/pytest_c3_pro$v.log 2>&1 || { grep -E "^E |FAILED" $O/pytest_c3_pro$v.log | head; exit 1; }
  echo "pro=$v c3: $(tail -1 $O/pytest_c3_pro$v.log)"
done
