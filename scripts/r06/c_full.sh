#!/bin/bash
# round 6 checkpoint: the default bench (window 8, block Lanczos, calibration,
# box clocks), then the whole -m gpu suite and smoke()
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_c
mkdir -p $O
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], [round(x,3) for x in d['mode_product_ms_by_position']], d['roofline']['frac'], d['roofline']['traffic_source'], d['prologue_calibration_gbs'], d['prologue_calibration'], d['box'])
print('matvec', d['matvec']['ms'], 'block', d['block_matvec']['ms'], 'lanczos', d['lanczos']['basis'], d['lanczos']['ms_per_step'], d['lanczos']['mode_product_ms_by_position'])
print({k:(round(v.get('fit_ms'),2) if isinstance(v,dict) else v) for k,v in d['grief'].items()}, d['cpu_baseline']['value'])"
timeout -k 10 1500 python3 -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
tail -15 $O/pytest_gpu.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; tail -2 $O/smoke.log
