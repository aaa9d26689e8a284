#!/bin/bash
# the whole GPU suite on the final round-5 tree, then smoke()
set -o pipefail
O=gpurun_out/r05_ze
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
st=$?
tail -4 $O/pytest_gpu.log
[ $st -eq 0 ] || exit $st
timeout -k 10 90 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
