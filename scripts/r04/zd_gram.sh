#!/bin/bash
# C2 Gram (p = 1000, n = 1e5): split-K factor x grid variant
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r04_zd
mkdir -p $O
for v in "14 16" "14 21" "14 24" "14 12" "3 21" "3 24" "3 16"; do
  set -- $v
  GG_GEMM_TN=$1 GG_GEMM_SPLITK=$2 timeout -k 10 200 python -u bench_grief.py --configs C2 --repeats 3 --cpu off > $O/g_$1_$2.json 2> $O/g_$1_$2.err || { tail -20 $O/g_$1_$2.err; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$O/g_$1_$2.json') if l.startswith('{')][-1])
print('tn=$1 S=$2', round(d['stage_ms']['gram'],3), round(d['gram']['achieved'],1), 'fit', round(d['fit_ms'],3))"
done
