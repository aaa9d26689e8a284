#!/bin/bash
# the pair launch's non-temporal streams A/B: p loads / q stores
# (GG_BLK_EPI_NT) and X DMAs (GG_BLK_X_NT); bitwise test, then interleaved
# processes, fused CG at 200^4, and reads of the pair launch per variant
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_z
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_block.py -x -q --timeout 200 --timeout-method thread -k "nontemporal" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
for v in 00 10 01 11; do
  e=${v:0:1}; x=${v:1:1}
  GG_BLK_EPI_NT=$e GG_BLK_X_NT=$x timeout -k 10 200 python -u tools/block_bench.py --iters 30 --reps 3 --no-grid --no-matvec > $O/v${v}_$r.json 2> $O/v${v}_$r.err || { tail -5 $O/v${v}_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/v${v}_$r.json').read().strip().splitlines()[-1])
print('$r epi_nt $e x_nt $x', 'cg %.2f' % d['cg_block']['ms_per_iter'], [round(t,2) for t in d['cg_block']['launch_ms']])"
done
done
B="--steps 4 --warmup 2 --matvec 0 --lanczos 0 --grief off --cpu-baseline off"
GG_BLK_X_NT=1 timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-trace -d $O/rd_x -o rd --output-format csv -- python3 bench.py $B > $O/rd_x.log 2>&1 || { tail -5 $O/rd_x.log; exit 1; }
python3 tools/pmc_reads.py $O/rd_x
