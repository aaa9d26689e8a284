#!/bin/bash
# Round 2, session e: PMC passes (separate runs, kernel trace only):
#   mode-product HBM traffic by request size (reads / writes) at 200^4,
#   Gram GEMM wave-state / MFMA / LDS / L2 counters at n = 1e5, p = 5000.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02e
mkdir -p $O
B="python3 bench.py --steps 2 --warmup 1 --cpu-baseline off"
G="python3 tools/p2_kernels_bench.py --what gram --shapes 100000x5000"
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-trace -d $O/mp_rd -o run --output-format csv -- $B > $O/mp_rd.log 2>&1 || { tail -5 $O/mp_rd.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-trace -d $O/mp_wr -o run --output-format csv -- $B > $O/mp_wr.log 2>&1 || { tail -5 $O/mp_wr.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_LDS_BANK_CONFLICT --kernel-trace -d $O/gram_sq -o run --output-format csv -- $G > $O/gram_sq.log 2>&1 || { tail -5 $O/gram_sq.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --kernel-trace -d $O/gram_tcc -o run --output-format csv -- $G > $O/gram_tcc.log 2>&1 || { tail -5 $O/gram_tcc.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d $O/gram_sq2 -o run --output-format csv -- $G > $O/gram_sq2.log 2>&1 || { tail -5 $O/gram_sq2.log; exit 1; }
find $O -name "*counter_collection.csv" | head
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/eig_trace -o run --output-format csv -- python3 tools/p2_kernels_bench.py --what eig > $O/eig_trace.log 2>&1 || { tail -5 $O/eig_trace.log; exit 1; }
find $O/eig_trace -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200 | head -12
