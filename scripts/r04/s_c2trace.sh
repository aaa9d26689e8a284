#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r04_s
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- python3 -u bench_grief.py --configs C2 --repeats 2 --cpu off > $O/c2.jsonl 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/r04_s/c2/run_kernel_stats.csv')))
for r in rows[:25]:
    print(r['Name'][:110], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us avg', r['Percentage'])
PY
