#!/bin/bash
# Round-1 pass B: sharded virtual-rank tests, split-variant parity, variant
# A/B, bench with CPU baseline, rocprof kernel stats, then the full GPU suite.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-r1b}; shift
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh ${tag}_dist 300 python -m pytest tests/test_gpu_dist.py -q -p no:cacheprovider -x; rc=$?
ok $rc || exit $rc
GG_MP_VARIANT=3 scripts/gpu_step.sh ${tag}_kron_v3 300 python -m pytest tests/test_gpu_kron.py -q -p no:cacheprovider -x; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_modes 400 python tools/tune_mode.py 200 4 "0,3,4,5,6,1" 2; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_bench 400 python bench.py; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --cpu-baseline off; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_pytest 600 python -m pytest tests -m gpu -q -p no:cacheprovider; rc=$?
exit $rc
