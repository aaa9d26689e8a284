#!/bin/bash
# round 6 final measurement (the Lanczos closing pass timed apart) on the final kernel sources: the two PMC passes of
# the block CG (window 8 and derived r: 12 iterations so the last two carry the
# full window) -> profiles/r06/pmc_block.json; the default bench (which then
# reports roofline.traffic); a rocprofv3 kernel-trace + stats run of the same
# command
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r06_l
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_gpu_fold.py tests/test_gpu_block.py tests/test_gpu_c3.py -k "lanczos or slq" > $O/pytest_lz.log 2>&1 || { tail -30 $O/pytest_lz.log; exit 1; }
tail -3 $O/pytest_lz.log
B="--steps 2 --warmup 10 --matvec 0 --lanczos 0 --grief off --cpu-baseline off"
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-trace -d $O/rd -o rd --output-format csv -- python3 bench.py $B > $O/rd.log 2>&1 || { tail -5 $O/rd.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_WRREQ_64B_sum --kernel-trace -d $O/wr -o wr --output-format csv -- python3 bench.py $B > $O/wr.log 2>&1 || { tail -5 $O/wr.log; exit 1; }
python3 tools/pmc_block.py $O/rd $O/wr $O/pmc_block.json 8 1 && true
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
tail -c 1200 $O/bench.json
timeout -s KILL 600 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python3 bench.py > $O/bench_traced.json 2> $O/bench_traced.err || { tail -5 $O/bench_traced.err; exit 1; }
find $O/trace -name '*kernel_stats*'
