#!/bin/bash
# Round 2, session b: fusion-layout tests + A/B of the fused-CG layouts at 200^4,
# GRIEF fits with the p-system PCG leg.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kron.py -m gpu -x -v --timeout 200 --timeout-method thread -k "fusion or repair" > $O/pytest_fusion.log 2>&1 || { tail -20 $O/pytest_fusion.log; exit 1; }
tail -3 $O/pytest_fusion.log
for rep in 1 2; do
  for f in 0 1 2; do
    timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --cpu-baseline off --fusion $f > $O/bench_f${f}_r${rep}.json 2>> $O/bench.err || exit $?
    python -c "import json;d=json.load(open('$O/bench_f${f}_r${rep}.json'));print('fusion',$f,'rep',$rep,round(d['value'],3),[round(x,2) for x in d['mode_product_ms_by_position']])"
  done
done
timeout -k 10 600 python -u bench_grief.py --configs C2,C4,C5 --repeats 2 --cpu off --cg > $O/bench_grief.jsonl 2> $O/bench_grief.err || exit $?
python - <<'PY'
import json
for l in open("gpurun_out/r02b/bench_grief.jsonl"):
    d=json.loads(l); print(d["config"]["workload"], round(d["fit_ms"],2), {k: round(v,2) for k,v in d["stage_ms"].items()}, d.get("p_system_cg"))
PY
