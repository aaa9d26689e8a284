#!/bin/bash
# A/B: the CG prologue with non-temporal loads / stores, interleaved processes.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r04_t${TAG:-}
mkdir -p $O
(rocm-smi --showuniqueid 2>&1 || true) | grep -i "unique id" > $O/box.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fold.py -k "nontemporal or lean" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2 3 4; do
  for nt in ${NTS:-0 1 3}; do
    GG_FOLD_PRO_NT=$nt timeout -k 10 180 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off --grief off --lanczos 0 --matvec 0 > $O/b${nt}_$i.json 2> $O/b${nt}_$i.err || { tail -20 $O/b${nt}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b${nt}_$i.json'));print('nt=$nt', round(d['ms_per_step'],2), [round(v,2) for v in d['mode_product_ms_by_position']])"
  done
done
cat $O/box.txt
