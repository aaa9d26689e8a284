#!/bin/bash
# three-role pair kernel: block tests, then 200^4 block bench NR 3 vs 2
set -o pipefail
O=gpurun_out/r05_i
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_block.py -x -v --timeout 120 --timeout-method thread > $O/pytest_block.log 2>&1
st=$?
tail -3 $O/pytest_block.log
if [ $st -ne 0 ]; then exit $st; fi
timeout -k 10 240 python -u tools/block_bench.py --reps 5 > $O/bench_nr3.json 2> $O/bench_nr3.err || exit 1
cat $O/bench_nr3.json
GG_BLK_PAIR_NR=2 timeout -k 10 240 python -u tools/block_bench.py --reps 5 --no-grid > $O/bench_nr2.json 2> $O/bench_nr2.err || exit 1
cat $O/bench_nr2.json
GG_BLK_PAIR_ABL=12 timeout -k 10 240 python -u tools/block_bench.py --reps 5 --no-grid --no-cg > $O/bench_abl12.json 2> $O/bench_abl12.err || exit 1
cat $O/bench_abl12.json
