#!/bin/bash
# Round 2, session h: eigensolver (rsq chain + pipelined Z) tests and phases,
# Phi writer (product form, LDS-transposed store) tests, P2 kernel timings with
# a kernel trace of potrf, memory-side cache probe, GRIEF bench, P1 bench with
# kernel-trace stats.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_grief.py tests/test_gpu_configs.py tests/test_gpu_compat.py tests/test_gpu_web.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_p2.log 2>&1; rc=$?
tail -2 $O/pytest_p2.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_p2.log | head -20; exit $rc; }
GG_EIG_PROF=1 timeout -k 10 120 python -u tools/p2_kernels_bench.py --what eig > $O/eig_prof.log 2>&1 || { tail -5 $O/eig_prof.log; exit 1; }
grep -E "\"eig\"" $O/eig_prof.log; grep "eig m=" $O/eig_prof.log | awk '!seen[$2]++'
timeout -k 10 120 python -u tools/mall_probe.py > $O/mall.jsonl 2>&1 || { tail -5 $O/mall.jsonl; exit 1; }
cat $O/mall.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_potrf -o run -- python -u tools/p2_kernels_bench.py --what potrf,potrs --shapes 100000x10000 > $O/potrf.jsonl 2> $O/potrf.err || { tail -5 $O/potrf.err; exit 1; }
cat $O/potrf.jsonl
timeout -k 10 600 python -u bench_grief.py --configs C2,C4,C5 --repeats 2 --cpu off > $O/bench_grief.jsonl 2> $O/bench_grief.err || { tail -5 $O/bench_grief.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r02h/bench_grief.jsonl"):
    d=json.loads(l); print(d["config"]["workload"], round(d["fit_ms"],2), {k: round(v,2) for k,v in d["stage_ms"].items()}, "phi frac", round(d["phi"]["frac"],3))
PY
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python -u bench.py --steps 5 --warmup 2 --cpu-baseline off > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
