#!/bin/bash
# the vendor library's FP64 SYRK / GEMM against gemm_tn_glds on the GRIEF Gram
# shapes (n = 1e5; p = 1000 / 5000 / 10^4), one process each
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r06_h
mkdir -p $O
timeout -k 10 300 ./tools/syrk_probe 3 > $O/syrk.jsonl 2> $O/syrk.err || { cat $O/syrk.err; exit 1; }
cat $O/syrk.jsonl
timeout -k 10 300 python3 tools/p2_kernels_bench.py --what gram --vendor > $O/gram.jsonl 2> $O/gram.err || { tail -5 $O/gram.err; exit 1; }
cat $O/gram.jsonl
