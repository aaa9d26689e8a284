#!/bin/bash
# Lanczos prologue variants: parity of the tridiagonal, then the bench leg
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r04_zf${TAG:-}
mkdir -p $O
timeout -k 10 300 python -u - > $O/parity.txt 2>&1 <<'PY' || { tail -20 $O/parity.txt; exit 1; }
import os, sys, numpy as np
sys.path.insert(0, '.')
import bench
import gp_grief_amd as gg
from gp_grief_amd import linalg
m, d = 200, 3
K, F = bench.grid_factors(m, d)
out = {}
for v in ("0", "1", "2", "3"):
    os.environ["GG_FOLD_LZ"] = v
    a, b = linalg.lanczos_tridiag(K, 0.01, 20, seed=1, probe=0)
    out[v] = (np.asarray(a), np.asarray(b))
for v in ("1", "2", "3"):
    ra = np.abs(out[v][0] - out["0"][0]).max() / np.abs(out["0"][0]).max()
    rb = np.abs(out[v][1] - out["0"][1]).max() / np.abs(out["0"][1]).max()
    print(v, ra, rb)
    assert ra < 1e-10 and rb < 1e-10
print("parity ok")
PY
cat $O/parity.txt | tail -4
for i in 1 2; do
  for v in ${VARS:-0 1 2 3}; do
    GG_FOLD_LZ=${v%e} GG_FOLD_LZE=$([ "${v%e}" != "$v" ] && echo 1 || echo 0) timeout -k 10 240 python -u bench.py --steps 2 --warmup 1 --cpu-baseline off --grief off --lanczos 30 --matvec 0 > $O/b${v}_$i.json 2> $O/b${v}_$i.err || { tail -20 $O/b${v}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b${v}_$i.json'))['lanczos'];print('lz=$v', round(d['ms_per_step'],3), [round(v,2) for v in d['mode_product_ms_by_position']])"
  done
done
