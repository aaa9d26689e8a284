#!/bin/bash
# Round 2, session p: subset eigensolver path (bisection + inverse iteration)
# for the GRIEF setup: tests, P2 suite, GRIEF bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02p
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_grief.py -m gpu -x -v --timeout 120 --timeout-method thread -k "subset" > $O/pytest_subset.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" $O/pytest_subset.log | head -20
[ $rc -eq 0 ] || { grep -E "^E " $O/pytest_subset.log | head -30; exit $rc; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_grief.py tests/test_gpu_configs.py tests/test_gpu_compat.py tests/test_gpu_grief_dist.py tests/test_gpu_web.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_p2.log 2>&1; rc=$?
tail -2 $O/pytest_p2.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_p2.log | head -20; exit $rc; }
timeout -k 10 600 python -u bench_grief.py --configs C2,C4,C5 --repeats 3 --cpu off > $O/bench_grief.jsonl 2> $O/bench_grief.err || { tail -5 $O/bench_grief.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r02p/bench_grief.jsonl"):
    d=json.loads(l); print(d["config"]["workload"], round(d["fit_ms"],2), {k: round(v,2) for k,v in d["stage_ms"].items()})
PY
