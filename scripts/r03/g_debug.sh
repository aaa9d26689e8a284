#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
for xd in 1 0; do
for ms in 40,36,10 24,20,16,18 40,36; do
GG_KRON_FOLD_MIN=8 GG_CG_XDEFER=$xd timeout -k 10 120 python -u tools/cg_debug.py $ms || exit 1
done
GG_KRON_FOLD=0 GG_CG_XDEFER=$xd timeout -k 10 120 python -u tools/cg_debug.py 40,36,10 || exit 1
done
