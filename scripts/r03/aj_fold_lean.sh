#!/bin/bash
# round 3: plain folded mode product, lean A addressing (variant 8), B register
# double buffer (9), both (10; 11 / 12 at two waves per SIMD), interleaved in
# one process, output checked against variant 0
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03aj
mkdir -p $O
timeout -k 10 300 python -u tools/fold_variant_ab.py --variants ${VARS:-0,8,9,10,11,12,1} --rounds 3 > $O/ab.jsonl 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
cat $O/ab.jsonl
