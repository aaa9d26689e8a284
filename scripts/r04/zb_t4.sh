#!/bin/bash
# dense JT = 7 4x4-tail kernels: tests, then the parity per-rank probe
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r04_zb
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fold.py tests/test_gpu_kron.py tests/test_gpu_dist.py -k "t4 or parity or kron or fold" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 300 python -u tools/centro_shard_probe.py --worlds 2,4,8 --rotate 1 > $O/t4.jsonl 2> $O/t4.err || { tail -5 $O/t4.err; exit 1; }
GG_MP_NO_T4=1 timeout -k 10 300 python -u tools/centro_shard_probe.py --worlds 2,4,8 --rotate 1 > $O/not4.jsonl 2> $O/not4.err || { tail -5 $O/not4.err; exit 1; }
cat $O/t4.jsonl $O/not4.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['G'], d['rank'], round(d['ms_per_iteration'],3), [round(v,3) for v in d['launch_ms']])"
