#!/bin/bash
# SQ counters of the final block-basis CG launches at 200^4 (prologue =
# blk_mode_fast_kernel<6,3>, plain = <6,0>, pair + epilogue + side = blk_pair_lds_kernel)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_zj
mkdir -p $O
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace -d $O/sq -o run --output-format csv -- python3 tools/block_bench.py --no-matvec --iters 10 > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
python3 tools/sq_summary.py $O/sq prologue "blk_mode_fast_kernel<6, 3>" > $O/sq_summary.jsonl
python3 tools/sq_summary.py $O/sq plain "blk_mode_fast_kernel<6, 0>" >> $O/sq_summary.jsonl
python3 tools/sq_summary.py $O/sq pair blk_pair_lds_kernel >> $O/sq_summary.jsonl
python3 -c "
import json
for l in open('$O/sq_summary.jsonl'):
    r=json.loads(l); r.pop('per_launch'); print(json.dumps(r))"
