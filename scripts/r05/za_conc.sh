#!/bin/bash
# a share of the x side job on a concurrent stream beside the plain launch
# (GG_BLK_SIDE_CONC=<percent>): test, then interleaved processes at 200^4
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_za
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_block.py -x -q --timeout 200 --timeout-method thread -k "concurrent or nontemporal" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
for v in 0 20 35 50; do
  GG_BLK_SIDE_CONC=$v timeout -k 10 200 python -u tools/block_bench.py --iters 30 --reps 3 --no-grid --no-matvec > $O/c${v}_$r.json 2> $O/c${v}_$r.err || { tail -5 $O/c${v}_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/c${v}_$r.json').read().strip().splitlines()[-1])
print('$r conc $v', 'cg %.2f' % d['cg_block']['ms_per_iter'], [round(t,2) for t in d['cg_block']['launch_ms']])"
done
done
