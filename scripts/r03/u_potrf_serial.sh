#!/bin/bash
# round 3: Cholesky kernel trace with everything on one stream (isolated kernel times)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03u
mkdir -p $O
for pw in 256 512; do
GG_POTRF_LOOKAHEAD=0 GG_POTRF_PANEL=$pw timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt$pw -o run -- python3 -u tools/p2_kernels_bench.py --shapes 20000x10000 --what potrf > $O/kt$pw.log 2>&1 || { tail -5 $O/kt$pw.log; exit 1; }
done
echo done
