#!/bin/bash
# round 3: phase stamps of the Cholesky block chain (GG_POTRF_PROF) at C2/C4/C5 sizes,
# look-ahead on and off, plus a kernel trace of the p = 10^4 factor
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03p
mkdir -p $O
timeout -k 10 300 python -u tools/potrf_prof.py 1000,5000,10000 > $O/prof_la1.jsonl 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
cat $O/prof_la1.jsonl
timeout -k 10 300 python -u tools/potrf_prof.py 10000 --lookahead 0 --dump > $O/prof_la0.jsonl 2>> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
head -1 $O/prof_la0.jsonl
timeout -k 10 300 python -u tools/potrf_prof.py 10000 --dump > $O/prof_la1_dump.jsonl 2>> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 -u tools/p2_kernels_bench.py --shapes 20000x10000 --what potrf > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
echo done
