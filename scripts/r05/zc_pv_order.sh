#!/bin/bash
# the pair launch's epilogue operands issued behind the first fragments (this
# tree) against HEAD 131ba57 (_ab/, built in-tree): interleaved, fused CG at 200^4
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05_zc
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_block.py -x -q --timeout 200 --timeout-method thread -k "cg_vs_oracle or lds_kernel or nontemporal" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  timeout -k 10 200 python -u tools/block_bench.py --iters 30 --reps 3 --no-grid --no-matvec > $O/new_$r.json 2> $O/new_$r.err || { tail -5 $O/new_$r.err; exit 1; }
  timeout -k 10 200 python -u _ab/tools/block_bench.py --iters 30 --reps 3 --no-grid --no-matvec > $O/old_$r.json 2> $O/old_$r.err || { tail -5 $O/old_$r.err; exit 1; }
  python3 - $O $r <<'PY'
import json, sys
O, r = sys.argv[1], sys.argv[2]
for k in ("new", "old"):
    d = json.loads(open("%s/%s_%s.json" % (O, k, r)).read().strip().splitlines()[-1])
    print(r, k, "cg %.2f" % d["cg_block"]["ms_per_iter"], [round(t, 2) for t in d["cg_block"]["launch_ms"]])
PY
done
