#!/bin/bash
# round 3: plain folded mode products in isolation: timing, kernel trace, SQ counters
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03d
mkdir -p $O
rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -k 10 200 python -u tools/matvec_bench.py > $O/mv.json 2> $O/mv.err || { tail -5 $O/mv.err; exit 1; }
cat $O/mv.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/matvec_bench.py --reps 3 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc1 -o run -- python3 tools/matvec_bench.py --reps 2 > $O/pmc1.log 2>&1 || { tail -5 $O/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM --kernel-trace --output-format csv -d $O/pmc2 -o run -- python3 tools/matvec_bench.py --reps 2 > $O/pmc2.log 2>&1 || { tail -5 $O/pmc2.log; exit 1; }
echo done
