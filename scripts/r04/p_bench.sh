#!/bin/bash
# Prologue level after the 256-byte workspace alignment: 4 short CG-only
# processes, then the default bench line.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r04_p
mkdir -p $O
for i in 1 2 3 4; do
  timeout -k 10 180 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off --grief off --lanczos 0 --matvec 0 > $O/cg$i.json 2> $O/cg$i.err || { tail -20 $O/cg$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/cg$i.json'));print('$i', round(d['ms_per_step'],2), [round(v,2) for v in d['mode_product_ms_by_position']])"
done
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('default', round(d['value'],2), round(d['ms_per_step'],2), [round(v,2) for v in d['mode_product_ms_by_position']], d.get('lanczos',{}).get('ms_per_step'), d.get('matvec',{}).get('ms'))"
