#!/bin/bash
# pair launch read excess: L2 cache-policy A/B (GG_BLK_PAIR_ABL 64 side stream
# nt, 128 X DMAs nt, 4 no GEMM 2 k-loop), reads per launch + CG time
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_r
mkdir -p $O
B="--steps 4 --warmup 2 --matvec 0 --lanczos 0 --grief off --cpu-baseline off"
for v in 0 64 128 192 4; do
  GG_BLK_PAIR_ABL=$v timeout -k 10 180 python3 bench.py $B > $O/bench_$v.json 2> $O/bench_$v.err || { tail -5 $O/bench_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); print('abl $v', round(d['ms_per_step'],3), [round(t,3) for t in d['mode_product_ms_by_position']])"
  GG_BLK_PAIR_ABL=$v timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-trace -d $O/rd_$v -o rd --output-format csv -- python3 bench.py $B > $O/rd_$v.log 2>&1 || { tail -5 $O/rd_$v.log; exit 1; }
  python3 tools/pmc_reads.py $O/rd_$v
done
