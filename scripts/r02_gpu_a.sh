#!/bin/bash
# Round 2, session a: full GPU test suite (incl. C2-C5 config tests), bench with
# CPU baseline + Lanczos leg, rocprof kernel stats of the bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 400 --timeout-method thread ${PYTEST_EXTRA} \
  > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --lanczos 30 > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline off > $O/bench_prof.json 2> $O/bench_prof.err || exit $?
find $O/prof -name "*kernel_stats.csv" | head -3
