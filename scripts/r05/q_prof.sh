#!/bin/bash
# round-5 profiles of the default bench: rocprofv3 kernel trace + stats of the
# whole `bench.py` command, then the two PMC passes of the block CG launches
# (reads by request size, writes; separate runs, kernel trace only)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_q
mkdir -p $O
timeout -s KILL 900 rocprofv3 --kernel-trace --stats -d $O/trace -o bench -- python3 bench.py > $O/bench_traced.json 2> $O/bench_traced.err || { tail -5 $O/bench_traced.err; exit 1; }
tail -c 400 $O/bench_traced.json
B="--steps 4 --warmup 2 --matvec 0 --lanczos 0 --grief off --cpu-baseline off"
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-trace -d $O/rd -o rd --output-format csv -- python3 bench.py $B > $O/rd.log 2>&1 || { tail -5 $O/rd.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_WRREQ_64B_sum --kernel-trace -d $O/wr -o wr --output-format csv -- python3 bench.py $B > $O/wr.log 2>&1 || { tail -5 $O/wr.log; exit 1; }
python3 tools/pmc_block.py $O/rd $O/wr $O/pmc_block.json
