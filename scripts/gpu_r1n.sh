#!/bin/bash
# Re-validation of the restored tree: GPU parity suite, smoke, bench, P2 bench, kernel stats.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-r1n}
scripts/gpu_step.sh ${tag}_pytest 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread; rc=$?
[ $rc -eq 0 ] || exit $rc
scripts/gpu_step.sh ${tag}_smoke 300 python __graft_entry__.py smoke; rc=$?
[ $rc -eq 0 ] || exit $rc
scripts/gpu_step.sh ${tag}_bench 300 python bench.py; rc=$?
[ $rc -eq 0 ] || exit $rc
scripts/gpu_step.sh ${tag}_grief 400 python bench_grief.py; rc=$?
[ $rc -eq 0 ] || exit $rc
scripts/gpu_step.sh ${tag}_rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o run --output-format csv -- python bench.py --cpu-baseline off; rc=$?
exit $rc
