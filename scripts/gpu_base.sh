#!/bin/bash
# Parity + bench + kernel-trace profile of the current tree.
# usage: scripts/gpu_base.sh TAG
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-base}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh ${tag}_pytest 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider -x --timeout 120 --timeout-method thread; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_bench 300 python bench.py; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o run --output-format csv -- python bench.py --cpu-baseline off; rc=$?
exit $rc
