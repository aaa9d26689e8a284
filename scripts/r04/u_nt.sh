#!/bin/bash
# A/B: non-temporal streams of the CG epilogue / side launches, interleaved.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r04_u${TAG:-}
mkdir -p $O
(rocm-smi --showuniqueid 2>&1 || true) | grep -i "unique id" > $O/box.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_fold.py -k "nontemporal or lean" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2 3; do
  for v in ${VARS:-E0S0 E6S3 E6S0 E0S3}; do
    # v = E<epilogue mask>S<side mask>
    e=${v#E}; e=${e%%S*}; sm=${v##*S}; sm=${sm%%P*}
    pre=0; case $v in *P1) pre=1;; esac
    export GG_FOLD_EPI_NT=$e GG_FOLD_SIDE_NT=$sm GG_FOLD_EPI_PRE=$pre
    timeout -k 10 180 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off --grief off --lanczos 0 --matvec 0 > $O/b${v}_$i.json 2> $O/b${v}_$i.err || { tail -20 $O/b${v}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b${v}_$i.json'));print('$v', round(d['ms_per_step'],2), [round(v,2) for v in d['mode_product_ms_by_position']])"
  done
done
cat $O/box.txt
