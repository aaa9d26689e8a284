#!/bin/bash
# Round 2, session l: Cholesky with the last-arrival diagonal-block writer:
# look-ahead check at all sizes, P2 tests, timings and kernel trace.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02l
mkdir -p $O
timeout -k 10 300 python -u tools/potrf_check.py > $O/potrf_check.jsonl 2> $O/potrf_check.err || { tail -5 $O/potrf_check.err; exit 1; }
cat $O/potrf_check.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_grief.py tests/test_gpu_configs.py tests/test_gpu_compat.py tests/test_gpu_grief_dist.py tests/test_gpu_web.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_p2.log 2>&1; rc=$?
tail -2 $O/pytest_p2.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_p2.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/p2_kernels_bench.py --what potrf,potrs --vendor --shapes 100000x1000,100000x5000,100000x10000 > $O/potrf.jsonl 2> $O/potrf.err || { tail -5 $O/potrf.err; exit 1; }
cat $O/potrf.jsonl
GG_POTRF_LOOKAHEAD=0 timeout -k 10 300 python -u tools/p2_kernels_bench.py --what potrf --shapes 100000x10000 > $O/potrf_nola.jsonl 2> $O/potrf_nola.err || { tail -5 $O/potrf_nola.err; exit 1; }
cat $O/potrf_nola.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_potrf -o run -- python -u tools/p2_kernels_bench.py --what potrf --shapes 100000x10000 > $O/potrf_prof.jsonl 2> $O/potrf_prof.err || { tail -5 $O/potrf_prof.err; exit 1; }
timeout -k 10 600 python -u bench_grief.py --configs C2,C4,C5 --repeats 2 --cpu off > $O/bench_grief.jsonl 2> $O/bench_grief.err || { tail -5 $O/bench_grief.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r02l/bench_grief.jsonl"):
    d=json.loads(l); print(d["config"]["workload"], round(d["fit_ms"],2), {k: round(v,2) for k,v in d["stage_ms"].items()})
PY
