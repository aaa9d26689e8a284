#!/bin/bash
# LDS-ring pair kernel: block tests, then 200^4 block matvec / CG with the
# LDS pair kernel on and off
set -o pipefail
O=gpurun_out/r05_e
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_block.py -x -v --timeout 120 --timeout-method thread > $O/pytest_block.log 2>&1
st=$?
tail -5 $O/pytest_block.log
if [ $st -ne 0 ]; then exit $st; fi
timeout -k 10 240 python -u tools/block_bench.py --reps 5 > $O/bench_lds.json 2> $O/bench_lds.err || exit 1
cat $O/bench_lds.json
GG_BLK_PAIR_LDS=0 timeout -k 10 240 python -u tools/block_bench.py --reps 5 --no-grid > $O/bench_reg.json 2> $O/bench_reg.err || exit 1
cat $O/bench_reg.json
