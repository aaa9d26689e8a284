#!/bin/bash
# Round 2, session zf: subset eigenvectors by in-place reflector back-transform (no Z,
# no GEMM) + batched LDS loads in the tridiagonalisation: eigen tests, phase
# stamps, GRIEF setup times.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02zf
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kron.py tests/test_gpu_grief.py -m gpu -x -q --timeout 120 --timeout-method thread -k "eig or schur or subset or svd or grief or logdet" > $O/pytest_eig.log 2>&1 || { grep -E "^E |FAILED" $O/pytest_eig.log | head -20; exit 1; }
tail -1 $O/pytest_eig.log
GG_EIG_PROF=1 timeout -k 10 120 python -u tools/p2_kernels_bench.py --what eig > $O/eig_prof.log 2>&1 || { tail -5 $O/eig_prof.log; exit 1; }
grep -E '"what"' $O/eig_prof.log; grep -m1 "m=128" $O/eig_prof.log; grep -m1 "m=200" $O/eig_prof.log
for c in C2 C4 C5; do timeout -k 10 120 python -u tools/setup_profile.py $c 5 >> $O/setup_profile.jsonl 2>> $O/setup.err || exit $?; done
cat $O/setup_profile.jsonl
