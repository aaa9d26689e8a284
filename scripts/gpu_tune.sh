#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-tune}; shift
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh ${tag}_kron 600 python -m pytest tests/test_gpu_kron.py -q -p no:cacheprovider -x; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_modes 600 python tools/tune_mode.py 200 4 "${1:-0,3,4}" 2; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_grief 900 python -m pytest tests/test_gpu_grief.py -q -p no:cacheprovider; rc=$?
exit $rc
