#!/bin/bash
# round 6: within-box spread of the CG bench and the driver's W = 5 against
# the default W = 8 (three interleaved pairs, CG leg only)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_r
mkdir -p $O
for rep in 1 2 3; do
for w in 5 8; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup $w --matvec 0 --lanczos 0 --grief off --cpu-baseline off > $O/bench_w${w}_$rep.json 2> $O/bench_w${w}_$rep.err || { tail -5 $O/bench_w${w}_$rep.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_w${w}_$rep.json').read().strip().splitlines()[-1])
print('W=$w rep=$rep', round(d['value'],3), round(d['ms_per_step'],3), [round(x,3) for x in d['mode_product_ms_by_position']], round(d['prologue_calibration']['ms'],3), d['box']['gpu'].get('serial'))"
done
done
