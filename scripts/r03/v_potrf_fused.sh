#!/bin/bash
# round 3: fused newest in-panel term + side-stream in-panel updates + 3-per-CU update kernel
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03v
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_grief.py -m gpu -x -q -k "cholesky" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -20; exit $rc; }
GG_POTRF_PANEL=512 timeout -k 10 300 python -u -m pytest tests/test_gpu_grief.py -m gpu -x -q -k "cholesky" --timeout 120 --timeout-method thread > $O/pytest512.log 2>&1; rc=$?
tail -1 $O/pytest512.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest512.log | head -20; exit $rc; }
: > $O/ab.jsonl
for pw in 256 512; do
 for la in 1 0; do
  GG_POTRF_PANEL=$pw GG_POTRF_LOOKAHEAD=$la timeout -k 10 300 python -u tools/p2_kernels_bench.py --shapes 20000x1000,20000x5000,20000x10000 --what potrf > $O/t.jsonl 2> $O/t.err || { tail -5 $O/t.err; exit 1; }
  python -c "
import json
for l in open('$O/t.jsonl'):
    d=json.loads(l); d['panel']=$pw; d['lookahead']=$la; print(json.dumps(d))" >> $O/ab.jsonl
 done
done
cat $O/ab.jsonl
for pw in 256 512; do
GG_POTRF_PANEL=$pw timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt$pw -o run -- python3 -u tools/p2_kernels_bench.py --shapes 20000x10000 --what potrf > $O/kt$pw.log 2>&1 || { tail -5 $O/kt$pw.log; exit 1; }
GG_POTRF_LOOKAHEAD=0 GG_POTRF_PANEL=$pw timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kts$pw -o run -- python3 -u tools/p2_kernels_bench.py --shapes 20000x10000 --what potrf > $O/kts$pw.log 2>&1 || { tail -5 $O/kts$pw.log; exit 1; }
done
echo done
