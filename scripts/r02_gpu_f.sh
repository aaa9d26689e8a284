#!/bin/bash
# Round 2, session f: eigensolver phase stamps; TN-GEMM (Gram) variants:
# correctness (GEMM / triangle / Cholesky tests) and timing per variant.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02f
mkdir -p $O
GG_EIG_PROF=1 timeout -k 10 120 python -u tools/p2_kernels_bench.py --what eig > $O/eig_prof.log 2>&1 || { tail -5 $O/eig_prof.log; exit 1; }
grep -E "eig m=|\"eig\"" $O/eig_prof.log
for v in 1 2 3 4 5 0; do
  GG_GEMM_TN=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_grief.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or cholesky or fixtures_model" > $O/pytest_tn$v.log 2>&1 || { echo "variant $v FAILED"; tail -30 $O/pytest_tn$v.log; exit 1; }
  echo "variant $v tests: $(tail -1 $O/pytest_tn$v.log)"
  GG_GEMM_TN=$v timeout -k 10 300 python -u tools/p2_kernels_bench.py --what gram > $O/gram_tn$v.jsonl 2>> $O/gram.err || exit $?
  python -c "import json;[print('variant $v', json.loads(l)['p'], round(json.loads(l)['ms'],2), round(json.loads(l)['tflops'],1)) for l in open('$O/gram_tn$v.jsonl')]"
done
