#!/bin/bash
# round 3: every P2 GPU test after the setup / tables changes, GRIEF fits
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03ab
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_grief.py tests/test_gpu_configs.py tests/test_gpu_compat.py tests/test_gpu_grief_dist.py tests/test_gpu_web.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 600 python -u bench_grief.py --configs C2,C4,C5 --cpu off > $O/grief.jsonl 2> $O/grief.err || { tail -5 $O/grief.err; exit 1; }
python -c "
import json
for l in open('$O/grief.jsonl'):
    d=json.loads(l); print(d['config']['workload'], round(d['fit_ms'],3), {k: round(v,3) for k,v in d['stage_ms'].items()})"
echo done
