#!/bin/bash
# Round 2, session zb: TN Gram with fragment prefetch (11) and BK 16 (14) vs the
# launch-order kernel (3): GEMM tests, timings, L2 hit counters.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02zb
mkdir -p $O
for v in 11 14 3; do
  GG_GEMM_TN=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_grief.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or cholesky or fixtures_model" > $O/pytest_tn$v.log 2>&1 || { echo "variant $v FAILED"; grep -E "^E |FAILED" $O/pytest_tn$v.log | head; exit 1; }
  echo "variant $v tests: $(tail -1 $O/pytest_tn$v.log)"
  GG_GEMM_TN=$v timeout -k 10 300 python -u tools/p2_kernels_bench.py --what gram > $O/gram_tn$v.jsonl 2>> $O/gram.err || exit $?
  python -c "import json;[print('variant $v', json.loads(l)['p'], round(json.loads(l)['ms'],2), round(json.loads(l)['tflops'],1)) for l in open('$O/gram_tn$v.jsonl')]"
done
G="python -u tools/p2_kernels_bench.py --what gram --shapes 100000x10000"
