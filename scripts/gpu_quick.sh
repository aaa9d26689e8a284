#!/bin/bash
# Quick GPU iteration: kron tests + bench (no CPU baseline) + rocprof stats.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-quick}; shift
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh ${tag}_pytest 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_bench 600 python bench.py --steps 10 --warmup 2 --cpu-baseline off "$@"; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --cpu-baseline off "$@"; rc=$?
exit $rc
