#!/bin/bash
# round 3: Cholesky panel width A/B (GG_POTRF_PANEL) and look-ahead on/off
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03s
mkdir -p $O
: > $O/ab.jsonl
for pw in 256 512 768 1024; do
 for la in 1 0; do
  GG_POTRF_PANEL=$pw GG_POTRF_LOOKAHEAD=$la timeout -k 10 300 python -u tools/p2_kernels_bench.py --shapes 20000x5000,20000x10000 --what potrf > $O/t.jsonl 2> $O/t.err || { tail -5 $O/t.err; exit 1; }
  python -c "
import json
for l in open('$O/t.jsonl'):
    d=json.loads(l); d['panel']=$pw; d['lookahead']=$la; print(json.dumps(d))" >> $O/ab.jsonl
 done
done
cat $O/ab.jsonl
GG_POTRF_PANEL=512 timeout -k 10 300 python -u -m pytest tests/test_gpu_grief.py -m gpu -x -q -k "cholesky" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -20; exit $rc; }
GG_POTRF_PANEL=512 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 -u tools/p2_kernels_bench.py --shapes 20000x10000 --what potrf > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
echo done
