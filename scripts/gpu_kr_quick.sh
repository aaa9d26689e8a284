#!/bin/bash
# Khatri-Rao kernel iteration: KR tests, then the off-grid bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-krq}
scripts/gpu_step.sh ${tag}_kr 300 python -u -m pytest tests/test_gpu_kr.py -q -p no:cacheprovider --timeout 120 --timeout-method thread; rc=$?
[ $rc -eq 0 ] || exit $rc
scripts/gpu_step.sh ${tag}_offgrid 400 python bench_offgrid.py --cpu-baseline off; rc=$?
exit $rc
