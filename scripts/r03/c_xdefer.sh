#!/bin/bash
# round 3: folded sharded operator + deferred x update; parity then bench
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kron.py tests/test_gpu_fold.py tests/test_gpu_c3.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_kron.log 2>&1; rc=$?
tail -2 $O/pytest_kron.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest_kron.log | head -30; exit $rc; }
timeout -k 10 300 python -u bench.py --cpu-baseline off --lanczos 10 --grief off > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], [round(v,2) for v in d['mode_product_ms_by_position']], d['roofline']['frac'], d.get('lanczos'))"
GG_CG_XDEFER=0 timeout -k 10 300 python -u bench.py --cpu-baseline off --lanczos 0 --grief off > $O/bench_noxdefer.json 2> $O/bench2.err || { tail -5 $O/bench2.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_noxdefer.json')); print('no xdefer', d['value'], d['ms_per_step'], [round(v,2) for v in d['mode_product_ms_by_position']])"
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_dist.log 2>&1; rc=$?
tail -2 $O/pytest_dist.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest_dist.log | head -30; exit $rc; }
echo done
