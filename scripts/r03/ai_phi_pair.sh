#!/bin/bash
# round 3: Phi with column pairs (16-byte stores, one block per row strip, GG_PHI_PAIR=1) vs the 256-column kernel: P2 tests, then A/B of the GRIEF fits
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03ai
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_grief.py tests/test_gpu_configs.py tests/test_gpu_compat.py tests/test_gpu_grief_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -20; exit $rc; }
: > $O/ab.jsonl
for rep in 1 2; do
 for m in 1 0; do
  GG_PHI_PAIR=$m timeout -k 10 600 python -u bench_grief.py --configs C2,C5 --cpu off > $O/grief.jsonl 2> $O/grief.err || { tail -5 $O/grief.err; exit 1; }
  python -c "
import json
for l in open('$O/grief.jsonl'):
    d=json.loads(l); print(json.dumps({'pair': $m, 'rep': $rep, 'cfg': d['config']['workload'], 'fit_ms': round(d['fit_ms'],3), 'phi': round(d['stage_ms']['phi'],3), 'phi_gbs': round(d['phi']['achieved'],1)}))" >> $O/ab.jsonl
 done
done
cat $O/ab.jsonl
echo done
