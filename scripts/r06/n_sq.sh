#!/bin/bash
# round 6 final tree: one SQ / GRBM counter pass over the block CG's three
# launches (MFMA busy per SIMD, wave waits, effective clock)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r06_n
mkdir -p $O
B="--steps 4 --warmup 10 --matvec 0 --lanczos 0 --grief off --cpu-baseline off"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/sq -o sq --output-format csv -- python3 bench.py $B > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
for k in "blk_mode_fast_kernel<6, 5>" "blk_mode_fast_kernel<6, 0>" "blk_pair_lds_kernel<6, 3, 2, 1, 7>"; do
  python3 tools/sq_summary.py $O/sq "$k" "$k"
done > $O/sq_summary.jsonl
cat $O/sq_summary.jsonl
