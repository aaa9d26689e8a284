#!/bin/bash
# interleaved A/B on one box: k-step tiled slabs (this tree) against row-major
# slabs (_ab/: commit 7f1ee3d built in-tree), block matvec + fused CG, 3 rounds
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_u
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 200 python -u tools/block_bench.py --iters 30 --reps 5 --no-grid > $O/tiled_$r.json 2> $O/tiled_$r.err || { tail -5 $O/tiled_$r.err; exit 1; }
  timeout -k 10 200 python -u _ab/tools/block_bench.py --iters 30 --reps 5 --no-grid > $O/rowmajor_$r.json 2> $O/rowmajor_$r.err || { tail -5 $O/rowmajor_$r.err; exit 1; }
  python3 - $O $r <<'PY'
import json, sys
O, r = sys.argv[1], sys.argv[2]
for k in ("tiled", "rowmajor"):
    d = json.loads(open("%s/%s_%s.json" % (O, k, r)).read().strip().splitlines()[-1])
    print(r, k, "matvec %.2f" % d["block_matvec_ms"], [round(t, 2) for t in d["block_launch_ms"]],
          "cg %.2f" % d["cg_block"]["ms_per_iter"], [round(t, 2) for t in d["cg_block"]["launch_ms"]])
PY
done
