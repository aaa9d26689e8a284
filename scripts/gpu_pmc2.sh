#!/bin/bash
# HBM traffic of the dominant kernel: FETCH_SIZE / WRITE_SIZE in separate
# passes (kernel trace only) + the fetch calibration kernel, then the summary.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=${1:-pmc}
args="--steps 2 --warmup 1 --cpu-baseline off"
scripts/gpu_step.sh ${tag}_calib 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_${tag}_calib -o run --output-format csv -- tools/fetch_calib || exit $?
scripts/gpu_step.sh ${tag}_fetch 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_${tag}_fetch -o run --output-format csv -- python bench.py $args || exit $?
scripts/gpu_step.sh ${tag}_write 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_${tag}_write -o run --output-format csv -- python bench.py $args || exit $?
python tools/pmc_traffic.py gpurun_out/pmc_${tag}_fetch gpurun_out/pmc_${tag}_write gpurun_out/pmc_${tag}_calib "mode_product_kernel<13, 4, 3, 0, 3, true, 1, 2, 0>" gpurun_out/${tag}_traffic.json
