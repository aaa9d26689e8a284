#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh t4_tests 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh t4_modes 600 python tools/tune_mode.py 200 4 0,1,2,3,4 2; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh t4_bench 600 python bench.py --steps 10 --warmup 2 --cpu-baseline off; rc=$?
exit $rc
