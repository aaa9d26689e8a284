#!/bin/bash
# round 3: LDS-staged folded epilogue (GG_FOLD_STAGE=1) parity + A/B
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03h
mkdir -p $O
GG_FOLD_STAGE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_c3.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -30; exit $rc; }
for rep in 1 2; do
for st in 0 1; do
GG_FOLD_STAGE=$st timeout -k 10 300 python -u bench.py --cpu-baseline off --lanczos 10 --grief off > $O/bench_s$st.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_s$st.json')); print('stage $st', d['value'], d['ms_per_step'], [round(v,2) for v in d['mode_product_ms_by_position']], round(d['lanczos']['ms_per_step'],2))"
GG_FOLD_STAGE=$st timeout -k 10 100 python -u tools/matvec_bench.py --reps 5 || exit 1
done
done
echo done
