#!/bin/bash
# round 6 final tree: the whole -m gpu suite, smoke, the default bench (with
# roofline.traffic from the committed PMC passes) and the N = 2 one-card
# rehearsal of the multi-GPU line
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_m
mkdir -p $O
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
r=d['roofline']; lz=d['lanczos']
print(d['value'], d['ms_per_step'], [round(x,3) for x in d['mode_product_ms_by_position']], r['frac'], r['traffic'], r['traffic_source'], round(d['prologue_calibration']['ms'],3), d['box'].get('gfx_mhz'))
print('lanczos', lz['ms_per_step'], lz['closing_ms'], 'matvec', d['matvec']['ms'], 'block', d['block_matvec']['ms'])
print({k:(round(v.get('fit_ms'),2) if isinstance(v,dict) else v) for k,v in d['grief'].items()}, d['cpu_baseline']['value'])"
GG_BENCH_BACKEND=gloo-gpu timeout -k 10 600 python3 bench.py --gpus 2 --steps 5 --warmup 2 --grief off > $O/bench_n2.json 2> $O/bench_n2.err || { tail -5 $O/bench_n2.err; exit 1; }
tail -c 400 $O/bench_n2.json
timeout -k 10 1700 python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
tail -4 $O/pytest_gpu.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; tail -2 $O/smoke.log
