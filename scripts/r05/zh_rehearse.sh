#!/bin/bash
# (final tree) bench.py --gpus N rehearsed on one GPU: every rank on cuda:0, collectives over
# gloo (GG_BENCH_BACKEND=gloo-gpu); the lines must say "rehearsal".  N = 4 runs
# the sharded C4 GRIEF fit, N = 8 C5.
set -o pipefail
O=gpurun_out/r05_zh
mkdir -p $O
export PYTHONUNBUFFERED=1 GG_BENCH_BACKEND=gloo-gpu
for n in 2 4 8; do
  timeout -k 10 340 python -u bench.py --gpus $n --steps 5 --warmup 2 --matvec 0 --lanczos 0 > $O/n$n.json 2> $O/n$n.err || { tail -20 $O/n$n.err; exit 1; }
  python3 -c "
import json,sys
r=json.loads(open('$O/n$n.json').read().strip().splitlines()[-1])
print($n, r['value'], r['ms_per_step'], r['scaling'], r['backend'], r['physical_gpus'], r['config'].get('cg_basis'), r['roofline']['frac'], r['allreduce']['share_of_iteration'], r.get('fold_ms'), r.get('unfold_ms'), {k:(v.get('lml') if isinstance(v,dict) else v) for k,v in r.get('grief',{}).items()})"
done
