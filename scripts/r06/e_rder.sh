#!/bin/bash
# round 6: derived r -- block tests, then the CG bench A/B (derived vs stored
# r) interleaved, then the dist tests
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_e
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_gpu_block.py -k "rderive or window or cg" > $O/pytest_block.log 2>&1
tail -6 $O/pytest_block.log
B="--steps 20 --warmup 10 --matvec 0 --lanczos 0 --grief off --cpu-baseline off"
for rep in 1 2; do
for rd in 1 0; do
  GG_CG_RDERIVE=$rd timeout -k 10 300 python3 bench.py $B > $O/bench_rd${rd}_$rep.json 2> $O/bench_rd${rd}_$rep.err || { tail -5 $O/bench_rd${rd}_$rep.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_rd${rd}_$rep.json').read().strip().splitlines()[-1])
print('rd=$rd rep=$rep', round(d['value'],3), round(d['ms_per_step'],3), [round(x,3) for x in d['mode_product_ms_by_position']], d['config']['cg_r_derived'], round(d['prologue_calibration']['ms'],3), round(d['closing_ms'],2))"
done
done
timeout -k 10 900 python3 -u -m pytest -v --timeout 170 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_c3.py > $O/pytest_dist_c3.log 2>&1
tail -6 $O/pytest_dist_c3.log
