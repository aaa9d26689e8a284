#!/bin/bash
# Round 2, session y: diagonal-block inverses off the Cholesky chain (check,
# P2 tests, timing); SQ counters of the TN Gram kernel.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02y
mkdir -p $O
timeout -k 10 300 python -u tools/potrf_check.py 300,1000,5000,10000 > $O/potrf_check.jsonl 2> $O/potrf_check.err || { tail -5 $O/potrf_check.err; exit 1; }
cat $O/potrf_check.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_grief.py tests/test_gpu_configs.py tests/test_gpu_web.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_p2.log 2>&1; rc=$?
tail -2 $O/pytest_p2.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_p2.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/p2_kernels_bench.py --what potrf,potrs --shapes 100000x1000,100000x5000,100000x10000 > $O/potrf.jsonl 2> $O/potrf.err || { tail -5 $O/potrf.err; exit 1; }
cat $O/potrf.jsonl
G="python -u tools/p2_kernels_bench.py --what gram --shapes 100000x10000"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAIT_INST_LDS --kernel-trace -d $O/gram_sq -o run --output-format csv -- $G > $O/gram_sq.log 2>&1 || { tail -5 $O/gram_sq.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-trace -d $O/gram_sq2 -o run --output-format csv -- $G > $O/gram_sq2.log 2>&1 || { tail -5 $O/gram_sq2.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --kernel-trace -d $O/gram_tcc -o run --output-format csv -- $G > $O/gram_tcc.log 2>&1 || { tail -5 $O/gram_tcc.log; exit 1; }
echo done
