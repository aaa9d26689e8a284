#!/bin/bash
# Ring side-job kind: parity, then the CG bench with / without it.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r04_${TAG:-j}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ring.py tests/test_gpu_fold.py tests/test_gpu_c3.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -20; exit $rc; }
AB_VARIANTS=0,42 AB_ROUNDS=2 timeout -k 10 300 python -u tools/ring_ab.py > $O/ring_ab.jsonl 2> $O/ring_ab.err || { tail -5 $O/ring_ab.err; exit 1; }
cat $O/ring_ab.jsonl
for side in 0 1 0 1; do
  GG_FOLD_RING_SIDE=$side timeout -k 10 300 python -u bench.py --cpu-baseline off --grief off --lanczos 0 --matvec 0 --steps 20 > $O/bench_side$side.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_side$side.json')); print('side', $side, round(d['value'],3), round(d['ms_per_step'],2), [round(v,2) for v in d['mode_product_ms_by_position']])" | tee -a $O/side_ab.txt
done
