#!/bin/bash
# the whole GPU suite after the variant pruning (-s: the restart-penalty and
# forced-cancellation tests print their counts), then smoke()
set -o pipefail
O=gpurun_out/r05_t
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
st=$?
grep -E "restart penalty|forced cancellations|iterations \(oracle" $O/pytest_gpu.log
tail -4 $O/pytest_gpu.log
[ $st -eq 0 ] || exit $st
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
