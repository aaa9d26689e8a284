#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-r1e}; shift
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh ${tag}_calib_fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_${tag}_calib_fetch -o run --output-format csv -- tools/fetch_calib; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_calib_write 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_${tag}_calib_write -o run --output-format csv -- tools/fetch_calib; rc=$?
ok $rc || exit $rc
scripts/gpu_pmc.sh ${tag}; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_bench 400 python bench.py; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --cpu-baseline off; rc=$?
exit $rc
