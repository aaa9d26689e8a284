#!/bin/bash
# two-slab LDS pair kernel: block tests, 200^4 block bench (SPW 2 vs 1), ablation
set -o pipefail
O=gpurun_out/r05_g
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_block.py -x -v --timeout 120 --timeout-method thread > $O/pytest_block.log 2>&1
st=$?
tail -3 $O/pytest_block.log
if [ $st -ne 0 ]; then exit $st; fi
timeout -k 10 240 python -u tools/block_bench.py --reps 5 > $O/bench_spw2.json 2> $O/bench_spw2.err || exit 1
cat $O/bench_spw2.json
GG_BLK_PAIR_SPW=1 timeout -k 10 240 python -u tools/block_bench.py --reps 5 --no-grid --no-cg > $O/bench_spw1.json 2> $O/bench_spw1.err || exit 1
cat $O/bench_spw1.json
GG_BLK_PAIR_ABL=12 timeout -k 10 240 python -u tools/block_bench.py --reps 5 --no-grid --no-cg > $O/bench_abl12.json 2> $O/bench_abl12.err || exit 1
cat $O/bench_abl12.json
