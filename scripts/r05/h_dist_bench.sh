#!/bin/bash
# block sharding GPU tests (virtual ranks, 2 processes), then the default N = 1 bench
set -o pipefail
O=gpurun_out/r05_h
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -v -k "block or cg_comm" --timeout 300 --timeout-method thread > $O/pytest_dist_block.log 2>&1
st=$?
tail -3 $O/pytest_dist_block.log
if [ $st -ne 0 ]; then exit $st; fi
timeout -k 10 900 python -u bench.py > $O/bench_n1.json 2> $O/bench_n1.err
st=$?
tail -c 3000 $O/bench_n1.json
exit $st
