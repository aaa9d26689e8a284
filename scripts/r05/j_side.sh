#!/bin/bash
# x side job in the pair launch: block tests + dist block tests, then block CG with the
# side job in the pair launch vs in the second launch (GG_BLK_PAIR_ABL=32)
set -o pipefail
O=gpurun_out/r05_j
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests/test_gpu_block.py tests/test_gpu_dist.py -k "block or cg_comm" -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
st=$?
tail -3 $O/pytest.log
if [ $st -ne 0 ]; then exit $st; fi
timeout -k 10 240 python -u tools/block_bench.py --reps 5 --no-grid > $O/bench_side_pair.json 2> $O/bench_side_pair.err || exit 1
cat $O/bench_side_pair.json
GG_BLK_PAIR_ABL=32 timeout -k 10 240 python -u tools/block_bench.py --reps 5 --no-grid --no-matvec > $O/bench_side_mode.json 2> $O/bench_side_mode.err || exit 1
cat $O/bench_side_mode.json
