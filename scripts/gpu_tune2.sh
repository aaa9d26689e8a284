#!/bin/bash
# A/B of mode-product variants + parity of the tried variants on the kron tests.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-tune}; vars=${2:-0,8,9}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
for v in ${vars//,/ }; do
  GG_MP_VARIANT=$v scripts/gpu_step.sh ${tag}_kron_v$v 300 python -u -m pytest tests/test_gpu_kron.py -q -p no:cacheprovider -x --timeout 120 --timeout-method thread -k "matvec or cg"; rc=$?
  ok $rc || exit $rc
done
scripts/gpu_step.sh ${tag}_modes 500 python tools/tune_mode.py 200 4 "$vars" 2; rc=$?
exit $rc
