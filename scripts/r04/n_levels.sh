#!/bin/bash
# Prologue levels: per workspace allocation inside one process (with and
# without holding the previous one), then 4 fresh processes.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r04_n
mkdir -p $O
timeout -k 10 300 python -u tools/prologue_levels.py > $O/hold0.jsonl 2> $O/hold0.err || { tail -20 $O/hold0.err; exit 1; }
cat $O/hold0.jsonl
timeout -k 10 300 python -u tools/prologue_levels.py --hold 1 --pads 0,0,0,0,0,0,2,2,2,2 > $O/hold1.jsonl 2> $O/hold1.err || { tail -20 $O/hold1.err; exit 1; }
cat $O/hold1.jsonl
for i in 1 2 3 4; do
  timeout -k 10 200 python -u tools/prologue_levels.py --pads 0,0 > $O/proc$i.jsonl 2> $O/proc$i.err || { tail -20 $O/proc$i.err; exit 1; }
  cat $O/proc$i.jsonl
done
