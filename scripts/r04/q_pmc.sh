#!/bin/bash
# PMC traffic of the CG mode products only (the checkpoint's two passes).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r04_q
mkdir -p $O
(rocm-smi --showuniqueid --showclocks 2>&1 || true) > $O/box.txt
B="python3 bench.py --steps 4 --warmup 2 --cpu-baseline off --lanczos 0 --grief off --matvec 0"
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-trace -d $O/mp_rd -o run --output-format csv -- $B > $O/mp_rd.log 2>&1 || { tail -5 $O/mp_rd.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-trace -d $O/mp_wr -o run --output-format csv -- $B > $O/mp_wr.log 2>&1 || { tail -5 $O/mp_wr.log; exit 1; }
python3 tools/pmc_traffic.py $O/mp_rd $O/mp_wr $O/pmc_mode_product.json
mkdir -p profiles/r04 && cp $O/pmc_mode_product.json profiles/r04/pmc_mode_product.json
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off --lanczos 0 --grief off --matvec 0 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], [round(v,2) for v in d['mode_product_ms_by_position']], d['roofline']['traffic'], d['roofline']['traffic_source'])"
cat $O/box.txt | head -30
