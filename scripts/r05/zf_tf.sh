#!/bin/bash
# the block basis at the pair orders added late in round 5 (m = 104, 136, 168,
# d = 4): block vs grid K*x and fused CG per iteration
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_zg
mkdir -p $O
for m in 104 136 168; do
  timeout -k 10 300 python -u tools/block_bench.py --m $m --d 4 --iters 20 --reps 4 --grid-cg > $O/m$m.json 2> $O/m$m.err || { tail -5 $O/m$m.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/m$m.json').read().strip().splitlines()[-1])
print($m, 'block matvec %.2f' % d['block_matvec_ms'], 'grid matvec %.2f' % d['grid_matvec_ms'], 'cg block %.2f' % d['cg_block']['ms_per_iter'], 'cg grid', d.get('cg_grid', {}).get('ms_per_iter'))"
done
