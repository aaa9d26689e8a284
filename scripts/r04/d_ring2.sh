#!/bin/bash
# Ring kernel after the SGPR-addressing / no-copy rewrite: parity, A/B, SQ.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r04_${TAG:-d}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -20; exit $rc; }
AB_VARIANTS=${AB_VARIANTS:-0,1,5,2} AB_ROUNDS=2 timeout -k 10 300 python -u tools/ring_ab.py > $O/ring_ab.jsonl 2> $O/ring_ab.err || { tail -5 $O/ring_ab.err; exit 1; }
cat $O/ring_ab.jsonl
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
for v in ${SQ_VARIANTS:-1}; do
  GG_FOLD_RING=$v timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d $O/v$v -o run --output-format csv -- python3 tools/matvec_bench.py --reps 2 > $O/v$v.log 2>&1 || { tail -5 $O/v$v.log; exit 1; }
  python3 tools/sq_summary.py $O/v$v $v | tee -a $O/sq.jsonl
done
