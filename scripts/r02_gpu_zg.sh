#!/bin/bash
# Round 2, session zg: TN Gram with 128 x 256 tiles, accumulators held in AGPRs by
# inline-asm MFMA (11: BK 16 x 2, 12: BK 8 x 3, 13: BK 8 x 4) vs the default (3).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02zg
mkdir -p $O
for v in 11 12 13 3; do
  GG_GEMM_TN=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_grief.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or cholesky or fixtures_model" > $O/pytest_tn$v.log 2>&1 || { echo "variant $v FAILED"; grep -E "^E |FAILED" $O/pytest_tn$v.log | head; exit 1; }
  echo "variant $v tests: $(tail -1 $O/pytest_tn$v.log)"
  GG_GEMM_TN=$v timeout -k 10 300 python -u tools/p2_kernels_bench.py --what gram > $O/gram_tn$v.jsonl 2>> $O/gram.err || exit $?
  python -c "import json;[print('variant $v', json.loads(l)['p'], round(json.loads(l)['ms'],2), round(json.loads(l)['tflops'],1)) for l in open('$O/gram_tn$v.jsonl')]"
done
