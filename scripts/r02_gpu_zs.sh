#!/bin/bash
# Round 2, session zs: potrf look-ahead on CU-partitioned streams
# (GG_POTRF_CU_SPLIT = chain CUs per 32) vs shared CUs.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02zs
mkdir -p $O
GG_POTRF_CU_SPLIT=12 timeout -k 10 200 python -u -m pytest tests/test_gpu_grief.py -m gpu -x -q --timeout 100 --timeout-method thread -k "cholesky or fixtures" > $O/pytest.log 2>&1 || { grep -E "^E |FAILED" $O/pytest.log | head -20; tail -3 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in 0 8 12 16 20; do
  GG_POTRF_CU_SPLIT=$c timeout -k 10 200 python -u tools/p2_kernels_bench.py --what potrf --shapes 20000x1000,20000x5000,20000x10000 > $O/potrf_c$c.jsonl 2>> $O/p2.err || { tail -5 $O/p2.err; exit 1; }
  python -c "import json;[print('cu_split=$c', json.loads(l)['p'], round(json.loads(l)['ms'],2)) for l in open('$O/potrf_c$c.jsonl') if json.loads(l)['what']=='potrf']"
done
