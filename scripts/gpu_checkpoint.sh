#!/bin/bash
# Checkpoint on one MI355X: the whole GPU suite, smoke(), the default
# bench (with its CPU baseline) and a kernel-trace profile of the bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-checkpoint}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], [round(v,2) for v in d['mode_product_ms_by_position']], d['roofline']['frac'], d['roofline']['traffic'], d['cpu_baseline']['value'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python -u bench.py --steps 10 --warmup 2 --cpu-baseline off --lanczos 0 > $O/bench_prof.json 2> $O/bench_prof.err || { tail -5 $O/bench_prof.err; exit 1; }

# HBM traffic of the fused-CG mode products: two separate PMC passes (kernel
# trace only), reads by request size and writes (tools/pmc_traffic.py)
B="python3 bench.py --steps 2 --warmup 1 --cpu-baseline off --lanczos 0"
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-trace -d $O/mp_rd -o run --output-format csv -- $B > $O/mp_rd.log 2>&1 || { tail -5 $O/mp_rd.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-trace -d $O/mp_wr -o run --output-format csv -- $B > $O/mp_wr.log 2>&1 || { tail -5 $O/mp_wr.log; exit 1; }
python3 tools/pmc_traffic.py $O/mp_rd $O/mp_wr $O/pmc_mode_product.json
# GRIEF fits, stage-timed (C2 / C4 / C5)
timeout -k 10 600 python -u bench_grief.py --configs C2,C4,C5 --cpu off > $O/bench_grief.jsonl 2> $O/bench_grief.err || { tail -5 $O/bench_grief.err; exit 1; }
python -c "
import json
for l in open('$O/bench_grief.jsonl'):
    d=json.loads(l); print(d['config']['workload'], round(d['fit_ms'],2), {k: round(v,2) for k,v in d['stage_ms'].items()})"
echo checkpoint done
