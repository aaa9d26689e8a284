#!/bin/bash
# the CG prologue's output Y non-temporal too (GG_BLK_PRO_NT=2) against the
# default (1): bitwise test, interleaved processes, fused CG at 200^4
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_zi
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_block.py -x -q --timeout 200 --timeout-method thread -k "nontemporal" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
for v in 1 2; do
  GG_BLK_PRO_NT=$v timeout -k 10 200 python -u tools/block_bench.py --iters 30 --reps 3 --no-grid --no-matvec > $O/p${v}_$r.json 2> $O/p${v}_$r.err || { tail -5 $O/p${v}_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/p${v}_$r.json').read().strip().splitlines()[-1])
print('$r pro_nt $v', 'cg %.2f' % d['cg_block']['ms_per_iter'], [round(t,2) for t in d['cg_block']['launch_ms']])"
done
done
