#!/bin/bash
# Row-col Khatri-Rao matrix GPU tests, then the full GPU suite.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-r1q}
scripts/gpu_step.sh ${tag}_new 300 python -u -m pytest tests/test_gpu_rowcol_kr.py tests/test_gpu_kr.py -v -p no:cacheprovider --timeout 120 --timeout-method thread; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
scripts/gpu_step.sh ${tag}_pytest 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
scripts/gpu_step.sh ${tag}_offgrid 400 python bench_offgrid.py; rc=$?
[ $rc -eq 0 ] || exit $rc
scripts/gpu_step.sh ${tag}_rocprof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o run --output-format csv -- python bench_offgrid.py --cpu-baseline off; rc=$?
exit $rc
