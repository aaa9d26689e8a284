#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-r1g}; shift
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh ${tag}_pytest 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_modes 500 python tools/tune_mode.py 200 4 "0,1,3,5" 2; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_bench 400 python bench.py; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_rocprof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o run --output-format csv -- python bench.py; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_calib_fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_${tag}_calib_fetch -o run --output-format csv -- tools/fetch_calib; rc=$?
ok $rc || exit $rc
scripts/gpu_pmc.sh ${tag}; rc=$?
exit $rc
