#!/bin/bash
# Sharded-path GPU tests (virtual ranks + IPC processes), then the full GPU suite.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-dist}
scripts/gpu_step.sh ${tag}_dist 400 python -u -m pytest tests/test_gpu_dist.py -v -p no:cacheprovider -x --timeout 120 --timeout-method thread; rc=$?
[ $rc -eq 0 ] || exit $rc
scripts/gpu_step.sh ${tag}_pytest 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread; rc=$?
exit $rc
