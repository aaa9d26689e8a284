#!/bin/bash
# Round 2, session d: new eigensolver (tridiagonal + QL) tests and timing,
# GRIEF bench, and the gfx950 PMC counter list.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02d
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/pmc_list.txt 2>&1 || true
timeout -k 10 600 python -u -m pytest tests/test_gpu_kron.py tests/test_gpu_grief.py tests/test_gpu_c3.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 120 python -u tools/p2_kernels_bench.py --what eig > $O/eig.jsonl 2>&1 || exit $?
cat $O/eig.jsonl
GG_EIG=jacobi timeout -k 10 300 python -u tools/p2_kernels_bench.py --what eig > $O/eig_jacobi.jsonl 2>&1 || exit $?
timeout -k 10 600 python -u bench_grief.py --configs C2,C4,C5 --repeats 2 --cpu off > $O/bench_grief.jsonl 2> $O/bench_grief.err || { tail -5 $O/bench_grief.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r02d/bench_grief.jsonl"):
    d=json.loads(l); print(d["config"]["workload"], round(d["fit_ms"],2), {k: round(v,2) for k,v in d["stage_ms"].items()})
PY
