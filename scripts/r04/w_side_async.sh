#!/bin/bash
# The x side job on its own stream beside ring mode products: tests, then
# interleaved A/B against the side job inside the chunked kernels.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r04_w${TAG:-}
mkdir -p $O
(rocm-smi --showuniqueid 2>&1 || true) | grep -i "unique id" > $O/box.txt
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fold.py tests/test_gpu_kron.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for i in 1 2 3; do
  for v in 1 0; do
    GG_CG_SIDE_ASYNC=$v timeout -k 10 180 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off --grief off --lanczos 0 --matvec 0 > $O/b${v}_$i.json 2> $O/b${v}_$i.err || { tail -20 $O/b${v}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b${v}_$i.json'));print('async=$v', round(d['ms_per_step'],2), [round(v,2) for v in d['mode_product_ms_by_position']])"
  done
done
cat $O/box.txt
