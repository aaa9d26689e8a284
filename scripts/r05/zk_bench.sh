#!/bin/bash
# the default bench on the final tree (a second data point beside zd_final)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_zk
mkdir -p $O
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], [round(x,3) for x in d['mode_product_ms_by_position']], d['roofline']['frac'], d['roofline']['traffic'], d['roofline']['traffic_source'], d['matvec']['ms'], d['block_matvec']['ms'], d['lanczos']['ms_per_step'], {k:(round(v.get('fit_ms'),2) if isinstance(v,dict) else v) for k,v in d['grief'].items()})"
