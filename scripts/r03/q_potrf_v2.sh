#!/bin/bash
# round 3: the four-column block step (potrf_fac_kernel + potrf_upd_kernel):
# Cholesky tests, phase stamps, factor times vs the round-2 block step and vendor
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03q
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_grief.py -m gpu -x -q -k "cholesky" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/potrf_check.py 300,1000,2500,5000,10000 > $O/check.jsonl 2> $O/check.err || { tail -5 $O/check.err; exit 1; }
cat $O/check.jsonl
timeout -k 10 300 python -u tools/potrf_prof.py 1000,5000,10000 > $O/prof.jsonl 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
cat $O/prof.jsonl
timeout -k 10 300 python -u tools/p2_kernels_bench.py --shapes 20000x1000,20000x5000,20000x10000 --what potrf --vendor > $O/v2.jsonl 2> $O/v2.err || { tail -5 $O/v2.err; exit 1; }
GG_POTRF_V1=1 timeout -k 10 300 python -u tools/p2_kernels_bench.py --shapes 20000x1000,20000x5000,20000x10000 --what potrf > $O/v1.jsonl 2> $O/v1.err || { tail -5 $O/v1.err; exit 1; }
cat $O/v2.jsonl $O/v1.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 -u tools/p2_kernels_bench.py --shapes 20000x10000 --what potrf > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
echo done
