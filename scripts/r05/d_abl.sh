#!/bin/bash
# pair-kernel memory-stream ablation (diag): X from 16 slabs / Z to 16 slabs;
# then the block matvec + CG legs
set -o pipefail
O=gpurun_out/r05_d
mkdir -p $O
for a in 0 4 8 12; do
  GG_BLK_PAIR_ABL=$a timeout -k 10 120 python3 tools/block_bench.py --no-cg --no-grid --reps 5 > $O/abl$a.json 2> $O/abl$a.err || exit 1
  echo "abl=$a $(cat $O/abl$a.json)"
done


