#!/bin/bash
# split of the x side job between the second launch (GG_BLK_SIDE_PCT % of each
# half) and the pair launch; 30 CG iterations per setting, correctness first
set -o pipefail
O=gpurun_out/r05_n
mkdir -p $O
export PYTHONUNBUFFERED=1
GG_BLK_SIDE_PCT=30 timeout -k 10 300 python -u -m pytest tests/test_gpu_block.py -x -q -k "cg" --timeout 120 --timeout-method thread > $O/pytest_split30.log 2>&1 || { tail -20 $O/pytest_split30.log; exit 1; }
tail -2 $O/pytest_split30.log
for pct in 0 15 30 45 0; do
  GG_BLK_SIDE_PCT=$pct timeout -k 10 240 python -u tools/block_bench.py --iters 30 --no-grid --no-matvec > $O/pct$pct.json 2> $O/pct$pct.err || exit 1
  echo "pct $pct $(cat $O/pct$pct.json)"
done
