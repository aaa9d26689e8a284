#!/bin/bash
# the all-gather solution route of the block-sharded solve: the GPU
# distributed tests (virtual ranks + gloo processes) and an N = 2 rehearsal of
# the bench line that times both routes
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_i
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dist.py > $O/pytest_dist.log 2>&1 || { tail -30 $O/pytest_dist.log; exit 1; }
tail -3 $O/pytest_dist.log
GG_BENCH_BACKEND=gloo-gpu timeout -k 10 600 python3 bench.py --gpus 2 --steps 5 --warmup 2 --grief off > $O/bench_n2.json 2> $O/bench_n2.err || { tail -5 $O/bench_n2.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_n2.json').read().strip().splitlines()[-1])
print({k: d.get(k) for k in ('value','ms_per_step','fold_ms','unfold_ms','unfold_all_ms','solution_allreduce_ms','solution_allgather_ms')})"
