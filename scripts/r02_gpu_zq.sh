#!/bin/bash
# Round 2, session zq: potrf block kernel at 69 KB LDS + the look-ahead wide
# update on 2 workgroups per CU (GG_POTRF_WIDE_SLOTS 0 = old launch-order grid).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02zq
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_grief.py -m gpu -x -q --timeout 120 --timeout-method thread -k "cholesky or fixtures" > $O/pytest.log 2>&1 || { grep -E "^E |FAILED" $O/pytest.log | head -20; tail -3 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for w in 0 2 1 3 2; do
  GG_POTRF_WIDE_SLOTS=$w timeout -k 10 300 python -u tools/p2_kernels_bench.py --what potrf --shapes 20000x1000,20000x5000,20000x10000 > $O/potrf_w$w.jsonl 2>> $O/p2.err || { tail -5 $O/p2.err; exit 1; }
  python -c "import json;[print('wide_slots=$w', json.loads(l)['p'], round(json.loads(l)['ms'],2)) for l in open('$O/potrf_w$w.jsonl') if json.loads(l)['what']=='potrf']"
done
