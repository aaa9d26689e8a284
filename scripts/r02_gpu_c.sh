#!/bin/bash
# Round 2, session c: GRIEF fits (+ p-system PCG leg) and P2 dense-kernel
# microbenchmarks against the vendor library.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02c
mkdir -p $O
timeout -k 10 300 python -u tools/p2_kernels_bench.py --vendor > $O/p2_kernels.jsonl 2> $O/p2_kernels.err || { tail -5 $O/p2_kernels.err; exit 1; }
cat $O/p2_kernels.jsonl
timeout -k 10 600 python -u bench_grief.py --configs C2,C4,C5 --repeats 2 --cpu off --cg > $O/bench_grief.jsonl 2> $O/bench_grief.err || { tail -5 $O/bench_grief.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r02c/bench_grief.jsonl"):
    d=json.loads(l); print(d["config"]["workload"], round(d["fit_ms"],2), {k: round(v,2) for k,v in d["stage_ms"].items()}, d.get("p_system_cg"))
PY
