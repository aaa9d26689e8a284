#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-r1d}; shift
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh ${tag}_kron 300 python -m pytest tests/test_gpu_kron.py tests/test_gpu_dist.py -q -p no:cacheprovider -x; rc=$?
ok $rc || exit $rc
GG_MP_VARIANT=5 scripts/gpu_step.sh ${tag}_kron_v5 300 python -m pytest tests/test_gpu_kron.py -q -p no:cacheprovider -x; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_modes 500 python tools/tune_mode.py 200 4 "0,1,2,3,4,5" 2; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_bench 300 python bench.py --cpu-baseline off; rc=$?
exit $rc
