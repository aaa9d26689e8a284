#!/bin/bash
# Round 2, session i: pipelined fused-CG epilogue + split x side job: Kronecker
# / CG tests, then the P1 bench with a kernel trace.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kron.py tests/test_gpu_c3.py tests/test_gpu_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_kron.log 2>&1; rc=$?
tail -2 $O/pytest_kron.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_kron.log | head -20; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python -u bench.py --steps 10 --warmup 2 --cpu-baseline off > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['mode_product_ms_by_position'], d['passes_by_position'], d['roofline']['frac'], d['roofline']['traffic'])"
