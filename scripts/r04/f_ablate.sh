#!/bin/bash
# Ring kernel ablations (diagnostic variants 11-17: wrong results, timing only)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r04_f
mkdir -p $O
AB_VARIANTS=${AB_VARIANTS:-0,1,21,5,25,16,26} AB_ROUNDS=2 timeout -k 10 300 python -u tools/ring_ab.py > $O/ring_ab.jsonl 2> $O/ring_ab.err || { tail -5 $O/ring_ab.err; exit 1; }
cat $O/ring_ab.jsonl
