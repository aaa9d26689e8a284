#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r04_o
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py -k "fused or refusal or ipc" > $O/dist.log 2>&1 || { tail -40 $O/dist.log; exit 1; }
tail -3 $O/dist.log
timeout -k 10 300 python -u tools/shard_compute.py --reps 5 --recurrence fused > $O/shard.jsonl 2> $O/shard.err || { tail -20 $O/shard.err; exit 1; }
cat $O/shard.jsonl
bash scripts/r04/n_levels.sh
