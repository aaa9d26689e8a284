#!/bin/bash
# round 3: beta's r.q from the conjugacy identity (GG_CG_RQ=1, epilogue reads p only) vs r.q read in the epilogue: CG tests, then interleaved A/B
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03af
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_kron.py tests/test_gpu_c3.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -20; exit $rc; }
: > $O/ab.jsonl
for rep in 1 2 3; do
 for m in 1 0; do
  GG_CG_RQ=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline off --lanczos 0 --grief off > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python -c "
import json
d=json.load(open('$O/b.json')); print(json.dumps({'rq': $m, 'rep': $rep, 'value': d['value'], 'ms': d['ms_per_step'], 'pos': [round(v,2) for v in d['mode_product_ms_by_position']], 'cfg_rq': d['config'].get('cg_rq_identity')}))" >> $O/ab.jsonl
 done
done
cat $O/ab.jsonl
echo done
