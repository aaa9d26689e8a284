#!/bin/bash
# round 6: x_defer mode 3 (the x window) -- block tests, then the CG bench at
# windows 0 (mode 2 pairs) / 4 / 6 / 8, interleaved twice on one box
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_a
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_block.py > $O/pytest_block.log 2>&1 || { tail -30 $O/pytest_block.log; exit 1; }
tail -3 $O/pytest_block.log
B="--steps 20 --warmup 5 --matvec 0 --lanczos 0 --grief off --cpu-baseline off"
for rep in 1 2; do
for w in 0 4 6 8; do
  GG_CG_XWIN=$w timeout -k 10 300 python3 bench.py $B > $O/bench_w${w}_$rep.json 2> $O/bench_w${w}_$rep.err || { tail -5 $O/bench_w${w}_$rep.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_w${w}_$rep.json').read().strip().splitlines()[-1])
print('w=$w rep=$rep', round(d['value'],3), round(d['ms_per_step'],3), [round(x,3) for x in d['mode_product_ms_by_position']], d['config']['cg_x_window'], round(d['closing_ms'],2))"
done
done
