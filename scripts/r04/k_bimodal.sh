#!/bin/bash
# Prologue-launch bimodality: TCC read latency / DRAM credit stalls per launch
# position in several fresh processes (each draws its own level), plus one
# pass asking for the per-instance read-request counter.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r04_k
mkdir -p $O
B="python3 bench.py --steps 6 --warmup 2 --cpu-baseline off --lanczos 0 --grief off --matvec 0"
C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_sum"
for p in 1 2 3 4 5; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $O/p$p -o run --output-format csv -- $B > $O/p$p.json 2> $O/p$p.err || { tail -5 $O/p$p.err; exit 1; }
done
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_WRREQ --kernel-trace -d $O/inst -o run --output-format csv -- $B > $O/inst.json 2> $O/inst.err || { tail -5 $O/inst.err; exit 1; }
python3 tools/bimodal_summary.py $O > $O/summary.txt; cat $O/summary.txt
