#!/bin/bash
# SQ counters of the block-basis kernels (mode / pair) on the 200^4 block matvec
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_b
mkdir -p $O
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace -d $O/sq -o run --output-format csv -- python3 tools/block_bench.py --no-cg --no-grid --reps 3 > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
python3 tools/sq_summary.py $O/sq mode blk_mode > $O/sq_summary.jsonl
python3 tools/sq_summary.py $O/sq pair blk_pair >> $O/sq_summary.jsonl
cat $O/sq_summary.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); r.pop('per_launch'); print(json.dumps(r))"
