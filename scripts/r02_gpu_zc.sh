#!/bin/bash
# Round 2, session zc: chained multi-RHS triangular solve on MFMA: P2 tests,
# potrs / inverse_diag timings (chain vs blocked), GRIEF bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02zc
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_grief.py tests/test_gpu_configs.py tests/test_gpu_compat.py tests/test_gpu_web.py tests/test_gpu_grief_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_p2.log 2>&1; rc=$?
tail -2 $O/pytest_p2.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_p2.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/p2_kernels_bench.py --what potrs --shapes 100000x1000,100000x5000,100000x10000 > $O/potrs_chain.jsonl 2> $O/potrs_chain.err || { tail -5 $O/potrs_chain.err; exit 1; }
GG_TRSV_CHAIN=0 timeout -k 10 300 python -u tools/p2_kernels_bench.py --what potrs --shapes 100000x1000,100000x10000 > $O/potrs_blocked.jsonl 2> $O/potrs_blocked.err || { tail -5 $O/potrs_blocked.err; exit 1; }
cat $O/potrs_chain.jsonl $O/potrs_blocked.jsonl
timeout -k 10 600 python -u bench_grief.py --configs C2,C4,C5 --repeats 3 --cpu off > $O/bench_grief.jsonl 2> $O/bench_grief.err || { tail -5 $O/bench_grief.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r02zc/bench_grief.jsonl"):
    d=json.loads(l); print(d["config"]["workload"], round(d["fit_ms"],2), {k: round(v,2) for k,v in d["stage_ms"].items()})
PY
