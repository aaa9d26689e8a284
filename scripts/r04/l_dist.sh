#!/bin/bash
# Sharded CG: the fused recurrence (virtual ranks + IPC processes), then the
# bimodality diagnostic.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r04_l
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py > $O/dist.log 2>&1 || { tail -40 $O/dist.log; exit 1; }
tail -3 $O/dist.log
timeout -k 10 400 python -u tools/shard_compute.py --reps 5 > $O/shard.jsonl 2> $O/shard.err || { tail -20 $O/shard.err; exit 1; }
cat $O/shard.jsonl
bash scripts/r04/k_bimodal.sh
