#!/bin/bash
# Round 2, session k: Cholesky look-ahead debug (sizes x look-ahead on/off),
# eigensolver with the uniform QL chain (tests + phases).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02k
mkdir -p $O
timeout -k 10 300 python -u tools/potrf_check.py > $O/potrf_check.jsonl 2> $O/potrf_check.err || { tail -5 $O/potrf_check.err; exit 1; }
cat $O/potrf_check.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_kron.py tests/test_gpu_grief.py -m gpu -x -q --timeout 120 --timeout-method thread -k "eigensolver or schur or grid_gp or fixture or automobile or fd_gradient" > $O/pytest_eig.log 2>&1 || { tail -30 $O/pytest_eig.log; exit 1; }
echo "eig tests: $(tail -1 $O/pytest_eig.log)"
GG_EIG_PROF=1 timeout -k 10 120 python -u tools/p2_kernels_bench.py --what eig > $O/eig_prof.log 2>&1 || { tail -5 $O/eig_prof.log; exit 1; }
grep -E "\"eig\"" $O/eig_prof.log; grep "eig m=" $O/eig_prof.log | awk '!seen[$2]++'
