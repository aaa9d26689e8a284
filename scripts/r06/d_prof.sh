#!/bin/bash
# round 6: padded block-basis tests; block vs grid at 64^4 / 96^4 / 128^4;
# the block-shard per-rank probe at G = 1/2/4/8; PMC passes of the window-8
# CG; the default bench under a rocprofv3 kernel trace
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06_d
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_block.py tests/test_gpu_dist.py -k "padded or unavailable or info or device_parity or fallback" > $O/pytest_padded.log 2>&1
tail -4 $O/pytest_padded.log
for m in 64 96 128; do
  timeout -k 10 300 python3 tools/block_bench.py --m $m --d 4 --iters 20 --grid-cg >> $O/block_vs_grid.jsonl 2> $O/bb_$m.err || { tail -5 $O/bb_$m.err; exit 1; }
done
cat $O/block_vs_grid.jsonl
timeout -k 10 600 python3 tools/block_rank_probe.py > $O/block_rank_probe.jsonl 2> $O/probe.err || { tail -5 $O/probe.err; exit 1; }
cat $O/block_rank_probe.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['G'], d['rank'], round(d['ms_per_iteration'],3), [round(x,3) for x in d['launch_ms']], round(d['fold_ms'],2), round(d['unfold_ms'],2))"
B="--steps 4 --warmup 2 --matvec 0 --lanczos 0 --grief off --cpu-baseline off"
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-trace -d $O/rd -o rd --output-format csv -- python3 bench.py $B > $O/rd.log 2>&1 || { tail -5 $O/rd.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_WRREQ_64B_sum --kernel-trace -d $O/wr -o wr --output-format csv -- python3 bench.py $B > $O/wr.log 2>&1 || { tail -5 $O/wr.log; exit 1; }
python3 tools/pmc_block.py $O/rd $O/wr $O/pmc_block.json 8
timeout -s KILL 600 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python3 bench.py > $O/bench_traced.json 2> $O/bench_traced.err || { tail -5 $O/bench_traced.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_traced.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], [round(x,3) for x in d['mode_product_ms_by_position']], d['prologue_calibration_gbs'], d['prologue_calibration']['ms'], d['lanczos']['ms_per_step'])"
find $O/trace -name '*stats*'
