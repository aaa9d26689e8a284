#!/bin/bash
# Round 5, first block-basis run: GPU tests of the parity-block operator, then
# the 200^4 block matvec / CG timing.
set -o pipefail
mkdir -p gpurun_out/r05_a
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_block.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r05_a/pytest_block.log 2>&1
st=$?
tail -5 gpurun_out/r05_a/pytest_block.log
if [ $st -ne 0 ]; then exit $st; fi
timeout -k 10 300 python -u tools/block_bench.py > gpurun_out/r05_a/block_bench.json 2> gpurun_out/r05_a/block_bench.err
st=$?
cat gpurun_out/r05_a/block_bench.json
exit $st
