#!/bin/bash
# the whole GPU suite (round-end tier), then smoke()
set -o pipefail
O=gpurun_out/r05_k
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
st=$?
tail -15 $O/pytest_gpu.log
exit $st
