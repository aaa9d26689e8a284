#!/bin/bash
# k-step tiled slab layout: block tests, block matvec / CG, bench, read PMC
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05_s
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_block.py tests/test_gpu_dist.py -x -q -s --timeout 300 --timeout-method thread -k "block or Block or restart or ill_cond" > $O/pytest_block.log 2>&1 || { tail -30 $O/pytest_block.log; exit 1; }
grep -E "restart penalty|iterations \(oracle" $O/pytest_block.log; tail -2 $O/pytest_block.log
for r in 1 2; do
  timeout -k 10 240 python -u tools/block_bench.py --iters 30 --reps 5 > $O/bench_$r.json 2> $O/bench_$r.err || exit 1
  echo "run $r $(cat $O/bench_$r.json)"
done
B="--steps 4 --warmup 2 --matvec 0 --lanczos 0 --grief off --cpu-baseline off"
timeout -k 10 180 python3 bench.py $B > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('bench', round(d['ms_per_step'],3), [round(t,3) for t in d['mode_product_ms_by_position']])"
timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-trace -d $O/rd -o rd --output-format csv -- python3 bench.py $B > $O/rd.log 2>&1 || { tail -5 $O/rd.log; exit 1; }
python3 tools/pmc_reads.py $O/rd
