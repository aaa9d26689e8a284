#!/bin/bash
# side job A/B in reversed order (second launch first, then the pair launch),
# 30 CG iterations each, twice
set -o pipefail
O=gpurun_out/r05_m
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  GG_BLK_PAIR_ABL=32 timeout -k 10 240 python -u tools/block_bench.py --iters 30 --no-grid --no-matvec > $O/mode_$r.json 2> $O/mode_$r.err || exit 1
  echo "mode $r $(cat $O/mode_$r.json)"
  timeout -k 10 240 python -u tools/block_bench.py --iters 30 --no-grid --no-matvec > $O/pair_$r.json 2> $O/pair_$r.err || exit 1
  echo "pair $r $(cat $O/pair_$r.json)"
done
