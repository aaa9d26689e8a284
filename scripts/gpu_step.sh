#!/bin/bash
# Run one GPU step with its own time limit; record its exit code.
# usage: scripts/gpu_step.sh NAME SECONDS cmd...
# Exit codes 0/1 (e.g. pytest test failures) let the caller continue; anything
# else (fault/abort/segfault/timeout) makes the caller stop touching the GPU.
name=$1; shift; secs=$1; shift
mkdir -p gpurun_out
echo "== $name: $*" | tee -a gpurun_out/steps.log
timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
tail -5 "gpurun_out/$name.log"
exit $rc
