#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-r1f}; shift
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh ${tag}_kron 300 python -m pytest tests/test_gpu_kron.py tests/test_gpu_dist.py -q -p no:cacheprovider -x; rc=$?
ok $rc || exit $rc
GG_MP_VARIANT=6 scripts/gpu_step.sh ${tag}_kron_v6 300 python -m pytest tests/test_gpu_kron.py -q -p no:cacheprovider -x; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_modes 500 python tools/tune_mode.py 200 4 "0,6,7,8" 2; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_bench 400 python bench.py; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_rocprof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o run --output-format csv -- python bench.py; rc=$?
exit $rc
