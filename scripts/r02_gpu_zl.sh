#!/bin/bash
# Round 2, session zl: split-K Gram by default (S = 8) and diag(P^-1) through the
# recursive triangular inverse (gg_trtri): P2 tests, kernel timings, stage-timed fits.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02zl
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_grief.py tests/test_gpu_configs.py tests/test_gpu_grief_dist.py tests/test_gpu_web.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_p2.log 2>&1 || { grep -E "^E |FAILED" $O/pytest_p2.log | head -20; tail -3 $O/pytest_p2.log; exit 1; }
tail -1 $O/pytest_p2.log
timeout -k 10 300 python -u tools/p2_kernels_bench.py --what gram,potrf,potrs > $O/p2_kernels.jsonl 2>> $O/p2.err || { tail -5 $O/p2.err; exit 1; }
cat $O/p2_kernels.jsonl
timeout -k 10 600 python -u bench_grief.py --configs C2,C4,C5 --cpu off > $O/bench_grief.jsonl 2> $O/bench_grief.err || { tail -5 $O/bench_grief.err; exit 1; }
python -c "
import json
for l in open('$O/bench_grief.jsonl'):
    d=json.loads(l); print(d['config']['workload'], round(d['fit_ms'],2), {k: round(v,2) for k,v in d['stage_ms'].items()})"
