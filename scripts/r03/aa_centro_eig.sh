#!/bin/bash
# round 3: batched MFMA tables + centrosymmetric half-order eigenproblems in the GRIEF setup
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03aa
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_grief.py -k "centro or subset or grief" -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -20; exit $rc; }
for c in C2 C4 C5; do
  for v in 1 0; do
    GG_EIG_CENTRO=$v timeout -k 10 120 python -u tools/setup_profile.py $c 3 2>$O/setup.err | grep config | python -c "import sys,json; d=json.loads(sys.stdin.read()); d['centro']=$v; print(json.dumps(d))" >> $O/setup.jsonl || exit 1
  done
done
cat $O/setup.jsonl
timeout -k 10 600 python -u bench_grief.py --configs C2,C4,C5 --cpu off > $O/grief.jsonl 2> $O/grief.err || { tail -5 $O/grief.err; exit 1; }
python -c "
import json
for l in open('$O/grief.jsonl'):
    d=json.loads(l); print(d['config']['workload'], round(d['fit_ms'],3), {k: round(v,3) for k,v in d['stage_ms'].items()})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 -u bench_grief.py --configs C2 --cpu off > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
echo done
