#!/bin/bash
# Round 2, session q: pipelined layout-1 epilogue: Kronecker / CG tests, then
# the P1 bench with fusion layouts 0 and 1.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kron.py tests/test_gpu_c3.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_kron.log 2>&1; rc=$?
tail -2 $O/pytest_kron.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_kron.log | head -20; exit $rc; }
for f in 0 1; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline off --fusion $f > $O/bench_f$f.json 2> $O/bench_f$f.err || { tail -5 $O/bench_f$f.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_f$f.json')); print('fusion $f', d['value'], d['ms_per_step'], [round(v,2) for v in d['mode_product_ms_by_position']], d['passes_by_position'])"
done
for c in C2 C5; do
  timeout -k 10 120 python -u tools/setup_profile.py $c 3 2>> $O/setup.err | tee -a $O/setup.jsonl || exit 1
  GG_EIG_SUBSET=0 timeout -k 10 120 python -u tools/setup_profile.py $c 3 2>> $O/setup.err | tee -a $O/setup.jsonl || exit 1
done
