#!/bin/bash
# PMC passes (one counter group per pass, kernel trace only) over a short
# bench run: HBM traffic (FETCH_SIZE, WRITE_SIZE) and SQ stall breakdown.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-pmc}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
args="--steps 2 --warmup 1 --cpu-baseline off"
scripts/gpu_step.sh ${tag}_pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_${tag}_fetch -o run --output-format csv -- python bench.py $args; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_${tag}_write -o run --output-format csv -- python bench.py $args; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ${tag}_pmc_sq 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_${tag}_sq -o run --output-format csv -- python bench.py $args; rc=$?
exit $rc
