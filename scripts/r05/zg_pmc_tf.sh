#!/bin/bash
# the block CG's two PMC passes again on the final sources (the TF 3..5
# instantiations changed gg_kronb.hip's hash), then the new pair orders' timing
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05_zg
mkdir -p $O
B="--steps 4 --warmup 2 --matvec 0 --lanczos 0 --grief off --cpu-baseline off"
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-trace -d $O/rd -o rd --output-format csv -- python3 bench.py $B > $O/rd.log 2>&1 || { tail -5 $O/rd.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_WRREQ_64B_sum --kernel-trace -d $O/wr -o wr --output-format csv -- python3 bench.py $B > $O/wr.log 2>&1 || { tail -5 $O/wr.log; exit 1; }
python3 tools/pmc_block.py $O/rd $O/wr $O/pmc_block.json
scripts/r05/zf_tf.sh
