#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-r1c}; shift
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh ${tag}_dist 300 python -m pytest tests/test_gpu_dist.py -q -p no:cacheprovider -x; rc=$?
ok $rc || exit $rc
scripts/gpu_pmc.sh ${tag}; rc=$?
exit $rc
