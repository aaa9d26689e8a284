#!/bin/bash
# the GPU test files from test_gpu_dist on (t_full stopped there), smoke(),
# then the tiled / row-major A/B
set -o pipefail
O=gpurun_out/r05_v
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_fold.py tests/test_gpu_grief.py tests/test_gpu_grief_dist.py tests/test_gpu_kr.py tests/test_gpu_kron.py tests/test_gpu_ring.py tests/test_gpu_rowcol_kr.py tests/test_gpu_web.py -m gpu -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
st=$?
grep -E "restart penalty|forced cancellations|iterations \(oracle" $O/pytest_gpu.log
tail -3 $O/pytest_gpu.log
[ $st -eq 0 ] || exit $st
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
scripts/r05/u_tile_ab.sh
