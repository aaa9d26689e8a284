#!/bin/bash
# the pair launch with the second half of its grid started later
# (GG_BLK_PAIR_STAGGER = s_sleep(127) count): block matvec + fused CG at 200^4
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_zb
mkdir -p $O
for r in 1 2; do
for v in 0 5 10 20; do
  GG_BLK_PAIR_STAGGER=$v timeout -k 10 200 python -u tools/block_bench.py --iters 20 --reps 4 --no-grid > $O/s${v}_$r.json 2> $O/s${v}_$r.err || { tail -5 $O/s${v}_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/s${v}_$r.json').read().strip().splitlines()[-1])
print('$r stagger $v', 'matvec %.2f' % d['block_matvec_ms'], [round(t,2) for t in d['block_launch_ms']], 'cg %.2f' % d['cg_block']['ms_per_iter'], [round(t,2) for t in d['cg_block']['launch_ms']])"
done
done
