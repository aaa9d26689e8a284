#!/bin/bash
# round 6: the window's side-job streams non-temporal (GG_BLK_SIDE_NT=1) --
# the window tests under it, then the CG bench A/B interleaved (both orders)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_k
mkdir -p $O
GG_BLK_SIDE_NT=1 timeout -k 10 600 python3 -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_gpu_block.py -k "window" > $O/pytest_window_nt.log 2>&1 || { tail -30 $O/pytest_window_nt.log; exit 1; }
tail -3 $O/pytest_window_nt.log
B="--steps 20 --warmup 10 --matvec 0 --lanczos 0 --grief off --cpu-baseline off"
for rep in 1 2 3; do
for nt in 1 0; do
  [ $rep = 2 ] && nt=$((1 - nt))
  GG_BLK_SIDE_NT=$nt timeout -k 10 300 python3 bench.py $B > $O/bench_nt${nt}_$rep.json 2> $O/bench_nt${nt}_$rep.err || { tail -5 $O/bench_nt${nt}_$rep.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_nt${nt}_$rep.json').read().strip().splitlines()[-1])
print('side_nt=$nt rep=$rep', round(d['value'],3), round(d['ms_per_step'],3), [round(x,3) for x in d['mode_product_ms_by_position']], round(d['prologue_calibration']['ms'],3))"
done
done
