#!/bin/bash
# Batched finite-difference eigen-bases: GRIEF GPU tests, then the fd-gradient bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-r1u}
scripts/gpu_step.sh ${tag}_grief 400 python -u -m pytest tests/test_gpu_grief.py -q -p no:cacheprovider --timeout 120 --timeout-method thread; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
scripts/gpu_step.sh ${tag}_fdgrad 400 python bench_fdgrad.py; rc=$?
exit $rc
