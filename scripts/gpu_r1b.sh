#!/bin/bash
# Round-1 pass B: all GPU parity tests (incl. sharded virtual ranks), variant
# A/B, bench with CPU baseline, rocprof kernel stats.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-r1b}; shift
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh ${tag}_dist 300 python -m pytest tests/test_gpu_dist.py -q -p no:cacheprovider -x; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_pytest 900 python -m pytest tests -m gpu -q -p no:cacheprovider; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_modes 600 python tools/tune_mode.py 200 4 "0,1,4,5" 2; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_bench 900 python bench.py; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --cpu-baseline off; rc=$?
exit $rc
