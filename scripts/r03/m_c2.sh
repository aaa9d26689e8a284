#!/bin/bash
# round 3: C2 GRIEF fit kernels (tables rewrite, Gram split-K) -- trace + counters
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_grief.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 300 python -u bench_grief.py --configs C2,C5 --cpu off > $O/grief.jsonl 2> $O/grief.err || { tail -5 $O/grief.err; exit 1; }
python -c "
import json
for l in open('$O/grief.jsonl'):
    d=json.loads(l); print(d['config']['workload'], round(d['fit_ms'],2), {k: round(v,3) for k,v in d['stage_ms'].items()}, round(d['gram']['achieved'],1), round(d['phi']['frac'],3))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 -u bench_grief.py --configs C2 --cpu off --repeats 2 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-trace --output-format csv -d $O/pmc1 -o run -- python3 bench_grief.py --configs C2 --cpu off --repeats 1 > $O/pmc1.log 2>&1 || { tail -5 $O/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $O/pmc2 -o run -- python3 bench_grief.py --configs C2 --cpu off --repeats 1 > $O/pmc2.log 2>&1 || { tail -5 $O/pmc2.log; exit 1; }
echo done
