#!/bin/bash
# round 3: Cholesky default (unfused) vs panel 512 vs fused; then every P2 GPU test and the GRIEF fits
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03w
mkdir -p $O
: > $O/ab.jsonl
for v in default p512 fuse; do
  case $v in default) E="";; p512) E="GG_POTRF_PANEL=512";; fuse) E="GG_POTRF_FUSE=1";; esac
  env $E timeout -k 10 300 python -u tools/p2_kernels_bench.py --shapes 20000x1000,20000x5000,20000x10000 --what potrf > $O/t.jsonl 2> $O/t.err || { tail -5 $O/t.err; exit 1; }
  python -c "
import json
for l in open('$O/t.jsonl'):
    d=json.loads(l); d['variant']='$v'; print(json.dumps(d))" >> $O/ab.jsonl
done
cat $O/ab.jsonl
timeout -k 10 900 python -u -m pytest tests/test_gpu_grief.py tests/test_gpu_configs.py tests/test_gpu_web.py tests/test_gpu_grief_dist.py tests/test_gpu_compat.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 600 python -u bench_grief.py --configs C2,C4,C5 --cpu off > $O/grief.jsonl 2> $O/grief.err || { tail -5 $O/grief.err; exit 1; }
python -c "
import json
for l in open('$O/grief.jsonl'):
    d=json.loads(l); print(d['config']['workload'], round(d['fit_ms'],2), {k: round(v,3) for k,v in d['stage_ms'].items()})"
echo done
