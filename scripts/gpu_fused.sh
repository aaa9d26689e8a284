#!/bin/bash
# Fused-CG check: kron GPU tests, then bench fused + textbook, rocprof of fused.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-fused}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh ${tag}_pytest 400 python -u -m pytest tests/test_gpu_kron.py -v -p no:cacheprovider -x --timeout 120 --timeout-method thread; rc=$?
[ $rc -eq 0 ] || exit $rc
scripts/gpu_step.sh ${tag}_bench 300 python bench.py --cpu-baseline off; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_bench_text 300 python bench.py --cpu-baseline off --recurrence textbook; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o run --output-format csv -- python bench.py --cpu-baseline off; rc=$?
exit $rc
