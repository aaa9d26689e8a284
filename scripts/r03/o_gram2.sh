#!/bin/bash
# round 3: XCD-slab split-K Gram as the default: P2 tests, Gram at C2/C4/C5, fits
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03o
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_grief.py tests/test_gpu_configs.py tests/test_gpu_web.py tests/test_gpu_grief_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -20; exit $rc; }
: > $O/gram.jsonl
for tn in 3 14; do
  GG_GEMM_TN=$tn timeout -k 10 200 python -u tools/p2_kernels_bench.py --shapes 100000x1000,100000x5000,100000x10000 --what gram > $O/g.json 2> $O/g.err || { tail -5 $O/g.err; exit 1; }
  python -c "
import json
for l in open('$O/g.json'):
    d=json.loads(l); d.update(tn=$tn); print(json.dumps(d))" >> $O/gram.jsonl
done
cat $O/gram.jsonl
timeout -k 10 600 python -u bench_grief.py --configs C2,C4,C5 --cpu off > $O/grief.jsonl 2> $O/grief.err || { tail -5 $O/grief.err; exit 1; }
python -c "
import json
for l in open('$O/grief.jsonl'):
    d=json.loads(l); print(d['config']['workload'], round(d['fit_ms'],2), {k: round(v,3) for k,v in d['stage_ms'].items()}, round(d['gram']['achieved'],1))"
echo done
