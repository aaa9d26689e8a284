#!/bin/bash
# round 3: padding loads skipped; prologue KC A/B; PMC of the prologue
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fold.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -30; exit $rc; }
GG_FOLD_PRO_KC=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_fold.py -m gpu -x -q --timeout 200 --timeout-method thread -k "cg or lanczos" > $O/pytest_kc1.log 2>&1; rc=$?
tail -2 $O/pytest_kc1.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest_kc1.log | head -30; exit $rc; }
for rep in 1 2; do
for kc in 2 1; do
GG_FOLD_PRO_KC=$kc timeout -k 10 300 python -u bench.py --cpu-baseline off --lanczos 0 --grief off > $O/bench_kc$kc.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_kc$kc.json')); print('pro kc $kc', d['value'], d['ms_per_step'], [round(v,2) for v in d['mode_product_ms_by_position']])"
done
done
B="python3 bench.py --steps 4 --warmup 2 --cpu-baseline off --lanczos 0 --grief off"
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-trace -d $O/mp_rd -o run --output-format csv -- $B > $O/mp_rd.log 2>&1 || { tail -5 $O/mp_rd.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-trace -d $O/mp_wr -o run --output-format csv -- $B > $O/mp_wr.log 2>&1 || { tail -5 $O/mp_wr.log; exit 1; }
python3 tools/pmc_traffic.py $O/mp_rd $O/mp_wr $O/pmc_mode_product.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['calibration'], d['calibrated_on_own_pattern'])"
echo done
