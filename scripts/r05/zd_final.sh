#!/bin/bash
# round-5 final sources: the block CG's two PMC passes (-> profiles/r05/pmc_block.json,
# keyed to the sources' sha256), then the default bench (roofline.traffic from it)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05_zd
mkdir -p $O
B="--steps 4 --warmup 2 --matvec 0 --lanczos 0 --grief off --cpu-baseline off"
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-trace -d $O/rd -o rd --output-format csv -- python3 bench.py $B > $O/rd.log 2>&1 || { tail -5 $O/rd.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_WRREQ_64B_sum --kernel-trace -d $O/wr -o wr --output-format csv -- python3 bench.py $B > $O/wr.log 2>&1 || { tail -5 $O/wr.log; exit 1; }
python3 tools/pmc_block.py $O/rd $O/wr $O/pmc_block.json && cp $O/pmc_block.json profiles/r05/pmc_block.json
timeout -s KILL 600 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
tail -c 300 $O/bench.json
