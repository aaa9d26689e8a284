#!/bin/bash
# bench.py --gpus N (parity sharding) rehearsed on ONE GPU: N ranks share the
# card, collectives over gloo (the per-rank times are not the N-GPU ones)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r04_zc
mkdir -p $O
for N in 2 4 8; do
  GG_BENCH_BACKEND=gloo-gpu timeout -k 10 420 python -u bench.py --gpus $N --steps 5 --warmup 2 > $O/n$N.json 2> $O/n$N.err || { tail -30 $O/n$N.err; exit 1; }
  grep '^{' $O/n$N.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print($N, d['n_gpus'], round(d['value'],3), round(d['ms_per_step'],2), d['config']['exchange'], d['config']['local_factor_orders'], {k: round(v,3) for k,v in d.get('phase_ms_per_iteration',{}).items()})"
done
