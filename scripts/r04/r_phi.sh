#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r04_r
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_grief.py tests/test_gpu_configs.py > $O/grief.log 2>&1 || { tail -40 $O/grief.log; exit 1; }
tail -3 $O/grief.log
for t in 0 1; do
  GG_GRIEF_LOGTAB=$t timeout -k 10 300 python -u bench_grief.py --configs C2,C4,C5 --repeats 3 --cpu off > $O/bg$t.jsonl 2> $O/bg$t.err || { tail -20 $O/bg$t.err; exit 1; }
  python3 -c "
import json
for l in open('$O/bg$t.jsonl'):
    d=json.loads(l); s=d['stage_ms']; print('logtab=$t', d['config']['workload'], round(d['fit_ms'],3), 'phi', round(s['phi'],3), 'gram', round(s['gram'],3), 'chol', round(s['chol'],3), 'setup', round(s['setup'],3))"
done
