#!/bin/bash
# Round 4, first GPU pass: the new timed entry points + ADVICE prologue-shape
# test + the folded / C3 suites, then the default bench (isolated K*x and
# per-step Lanczos legs) without the CPU baseline.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r04_a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_c3.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 600 python -u bench.py --cpu-baseline off > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print('cg', round(d['value'],3), round(d['ms_per_step'],2), [round(v,2) for v in d['mode_product_ms_by_position']])
print('matvec', json.dumps(d['matvec']))
print('lanczos', json.dumps(d['lanczos']))
print('grief', {k: round(v['fit_ms'],2) for k, v in d['grief'].items()})"
