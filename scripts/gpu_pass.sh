#!/bin/bash
# Generic GPU pass: parity tests, smoke, peak microbench, bench, rocprof stats.
# usage: scripts/gpu_pass.sh TAG [bench args...]
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-pass}; shift
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh ${tag}_pytest 900 python -m pytest tests -m gpu -q -p no:cacheprovider; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_smoke 300 python __graft_entry__.py smoke; rc=$?
ok $rc || exit $rc
if [ -x tools/mfma_f64_peak ]; then
  scripts/gpu_step.sh ${tag}_peak 120 tools/mfma_f64_peak; rc=$?
  ok $rc || exit $rc
fi
scripts/gpu_step.sh ${tag}_bench 900 python bench.py "$@"; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_rocprof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --cpu-baseline off; rc=$?
exit $rc
