#!/bin/bash
# Off-grid prediction bench at the C3 grid + kernel stats.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-r1p}
scripts/gpu_step.sh ${tag}_offgrid 400 python bench_offgrid.py; rc=$?
[ $rc -eq 0 ] || exit $rc
scripts/gpu_step.sh ${tag}_rocprof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o run --output-format csv -- python bench_offgrid.py --cpu-baseline off; rc=$?
exit $rc
