#!/bin/bash
# Round 2, session zk: TN Gram split-K sweep continued (S = 8 .. 48) at C2 / C4 / C5.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02zk
mkdir -p $O
for S in 1 8 12 16 24 32 48; do
  GG_GEMM_SPLITK=$S timeout -k 10 300 python -u tools/p2_kernels_bench.py --what gram --shapes 100000x1000,100000x5000,100000x10000 > $O/gram_s$S.jsonl 2>> $O/gram.err || exit $?
  python -c "import json;[print('S=$S', json.loads(l)['p'], round(json.loads(l)['ms'],2), round(json.loads(l)['tflops'],1)) for l in open('$O/gram_s$S.jsonl')]"
done
