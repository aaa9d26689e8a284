#!/bin/bash
# round 6: the x window (mode 3) and the block-basis Lanczos -- the CG bench at
# windows 0 (mode 2 pairs) / 4 / 6 / 8 interleaved, the Lanczos leg block vs
# grid, then the block tests (a failure is reported, not fatal to the timings)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_b
mkdir -p $O
B="--steps 20 --warmup 5 --matvec 0 --lanczos 0 --grief off --cpu-baseline off"
for rep in 1 2; do
for w in 0 4 6 8; do
  GG_CG_XWIN=$w timeout -k 10 300 python3 bench.py $B > $O/bench_w${w}_$rep.json 2> $O/bench_w${w}_$rep.err || { tail -5 $O/bench_w${w}_$rep.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_w${w}_$rep.json').read().strip().splitlines()[-1])
print('w=$w rep=$rep', round(d['value'],3), round(d['ms_per_step'],3), [round(x,3) for x in d['mode_product_ms_by_position']], d['config']['cg_x_window'], round(d['closing_ms'],2))"
done
done
L="--steps 2 --warmup 1 --matvec 0 --lanczos 30 --grief off --cpu-baseline off"
for lz in 1 0 1; do
  GG_LZ_BASIS=$lz timeout -k 10 300 python3 bench.py $L > $O/bench_lz${lz}.json 2> $O/bench_lz${lz}.err || { tail -5 $O/bench_lz${lz}.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_lz${lz}.json').read().strip().splitlines()[-1])['lanczos']
print('lz=$lz', d['basis'], round(d['ms_per_step'],3), round(d['steady_ms_per_step'],3), [round(x,3) for x in d['mode_product_ms_by_position']], d.get('roofline',{}).get('frac_hbm'))"
done
timeout -k 10 900 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_block.py > $O/pytest_block.log 2>&1
tail -15 $O/pytest_block.log
