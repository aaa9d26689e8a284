#!/bin/bash
# pair launch ablations (timing only): 64 GEMM 2 without fragment loads, 128
# without the x side job, 192 both; block matvec + fused CG
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_w
mkdir -p $O
for r in 1 2; do
for v in 0 64 128 192; do
  GG_BLK_PAIR_ABL=$v timeout -k 10 200 python -u tools/block_bench.py --iters 20 --reps 4 --no-grid > $O/abl${v}_$r.json 2> $O/abl${v}_$r.err || { tail -5 $O/abl${v}_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/abl${v}_$r.json').read().strip().splitlines()[-1])
print('$r abl $v', 'matvec %.2f' % d['block_matvec_ms'], [round(t,2) for t in d['block_launch_ms']], 'cg %.2f' % d['cg_block']['ms_per_iter'], [round(t,2) for t in d['cg_block']['launch_ms']])"
done
done
