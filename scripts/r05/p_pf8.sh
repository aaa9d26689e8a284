#!/bin/bash
# plain pair kernel with 8 F_{d-2} fragments in flight in GEMM 2: block tests,
# the block matvec / CG twice
set -o pipefail
O=gpurun_out/r05_p
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_block.py -x -q --timeout 120 --timeout-method thread > $O/pytest_block.log 2>&1 || { tail -20 $O/pytest_block.log; exit 1; }
tail -2 $O/pytest_block.log
for r in 1 2; do
  timeout -k 10 240 python -u tools/block_bench.py --iters 30 --reps 5 > $O/bench_$r.json 2> $O/bench_$r.err || exit 1
  echo "run $r $(cat $O/bench_$r.json)"
done
