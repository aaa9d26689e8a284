#!/bin/bash
# Round 2, session zt: left-looking panel Cholesky (GG_POTRF_MODE=left: one
# large-K split GEMM per panel, no look-ahead) vs the right-looking look-ahead.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02zt
mkdir -p $O
GG_POTRF_MODE=left timeout -k 10 200 python -u -m pytest tests/test_gpu_grief.py -m gpu -x -q --timeout 100 --timeout-method thread -k "cholesky or fixtures" > $O/pytest.log 2>&1 || { grep -E "^E |FAILED" $O/pytest.log | head -20; tail -3 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for m in right left right left; do
  GG_POTRF_MODE=$m timeout -k 10 200 python -u tools/p2_kernels_bench.py --what potrf --shapes 20000x1000,20000x5000,20000x10000 > $O/potrf_$m.jsonl 2>> $O/p2.err || { tail -5 $O/p2.err; exit 1; }
  python -c "import json;[print('$m', json.loads(l)['p'], round(json.loads(l)['ms'],2), json.loads(l).get('rel_err')) for l in open('$O/potrf_$m.jsonl') if json.loads(l)['what']=='potrf']"
done
