#!/bin/bash
# Register-resident Cholesky diagonal blocks: full GPU suite, then the P2 bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-r1w}
scripts/gpu_step.sh ${tag}_pytest 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread; rc=$?
[ $rc -eq 0 ] || exit $rc
scripts/gpu_step.sh ${tag}_grief 400 python bench_grief.py --cpu off; rc=$?
exit $rc
