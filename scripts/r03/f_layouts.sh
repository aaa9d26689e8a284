#!/bin/bash
# round 3: fusion layout 1 on the folded epilogue; deferred x; layout A/B
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_kron.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -30; exit $rc; }
for rep in 1 2; do
for f in 0 1; do
timeout -k 10 300 python -u bench.py --cpu-baseline off --lanczos 0 --grief off --fusion $f > $O/bench_f$f.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_f$f.json')); print('fusion $f', d['value'], d['ms_per_step'], [round(v,2) for v in d['mode_product_ms_by_position']])"
done
done
echo done
