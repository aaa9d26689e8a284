#!/bin/bash
# round 3: block kernel at <= 168 VGPRs, wide update padded to two workgroups per CU
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03r
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_grief.py -m gpu -x -q -k "cholesky" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -20; exit $rc; }
: > $O/ab.jsonl
for wl in default 0 40000; do
  if [ $wl = default ]; then unset GG_POTRF_WIDE_LDS; else export GG_POTRF_WIDE_LDS=$wl; fi
  timeout -k 10 300 python -u tools/p2_kernels_bench.py --shapes 20000x1000,20000x5000,20000x10000 --what potrf > $O/t.jsonl 2> $O/t.err || { tail -5 $O/t.err; exit 1; }
  python -c "
import json
for l in open('$O/t.jsonl'):
    d=json.loads(l); d['wide_lds']='$wl'; print(json.dumps(d))" >> $O/ab.jsonl
done
unset GG_POTRF_WIDE_LDS
cat $O/ab.jsonl
timeout -k 10 300 python -u tools/potrf_prof.py 5000,10000 > $O/prof.jsonl 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
cat $O/prof.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 -u tools/p2_kernels_bench.py --shapes 20000x10000 --what potrf > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
echo done
