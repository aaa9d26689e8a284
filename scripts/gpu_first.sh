#!/bin/bash
# First GPU pass: parity tests, smoke, a short bench.
cd "${GRAFT_REPO_ROOT:-.}"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh smoke 300 python __graft_entry__.py smoke; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh bench_short 600 python bench.py --steps 5 --warmup 1 --cpu-baseline off; rc=$?
exit $rc
