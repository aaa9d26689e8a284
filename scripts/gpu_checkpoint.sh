#!/bin/bash
# Checkpoint on one MI355X: the whole GPU suite, smoke(), the PMC traffic of
# the CG mode products (taken first, so the bench reports it), the default
# bench (with its CPU baseline and GRIEF leg) and a kernel-trace profile of it.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-checkpoint}
mkdir -p $O
# which box / clocks (the prologue's slow level has followed the box)
(rocm-smi --showuniqueid --showclocks --showmeminfo vram 2>&1 || true) > $O/box.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
# HBM traffic of the fused-CG mode products: two separate PMC passes (kernel
# trace only), reads by request size and writes (tools/pmc_traffic.py)
B="python3 bench.py --steps 4 --warmup 2 --cpu-baseline off --lanczos 0 --grief off --matvec 0"
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-trace -d $O/mp_rd -o run --output-format csv -- $B > $O/mp_rd.log 2>&1 || { tail -5 $O/mp_rd.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-trace -d $O/mp_wr -o run --output-format csv -- $B > $O/mp_wr.log 2>&1 || { tail -5 $O/mp_wr.log; exit 1; }
python3 tools/pmc_traffic.py $O/mp_rd $O/mp_wr $O/pmc_mode_product.json
# the bench below reports these counters when they match its kernels
mkdir -p profiles/r04 && cp $O/pmc_mode_product.json profiles/r04/pmc_mode_product.json
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], [round(v,2) for v in d['mode_product_ms_by_position']], d['roofline']['frac'], d['roofline']['traffic'], d['cpu_baseline']['value'], d['lanczos']['ms_per_step'], {k: round(v['fit_ms'],2) for k, v in d['grief'].items()})"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 -u bench.py --steps 10 --warmup 2 --cpu-baseline off --lanczos 0 --grief off > $O/bench_prof.json 2> $O/bench_prof.err || { tail -5 $O/bench_prof.err; exit 1; }
echo checkpoint done
