#!/bin/bash
# Round 2, session zi: HBM streaming ceiling for the CG pass mixes (8 GiB vectors).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r02zi
mkdir -p $O
timeout -k 10 300 ./tools/hbm_stream_bench > $O/hbm_stream.jsonl 2> $O/hbm_stream.err || { tail -5 $O/hbm_stream.err; exit 1; }
cat $O/hbm_stream.jsonl
