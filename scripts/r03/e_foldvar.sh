#!/bin/bash
# round 3: plain folded mode product, launch-shape variants (GG_FOLD_VARIANT), interleaved
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p $O
: > $O/var.jsonl
for rep in 1 2; do
for v in 0 1 2 3 4 5 6 7; do
  GG_FOLD_VARIANT=$v timeout -k 10 120 python -u tools/matvec_bench.py --reps 5 >> $O/var.jsonl 2> $O/err_$v.log || { tail -5 $O/err_$v.log; exit 1; }
done
done
cat $O/var.jsonl
