#!/bin/bash
# round 3: kernel-trace durations of the CG launches with each r.q source (rocprofv3 --kernel-trace --stats)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03ag
mkdir -p $O
for m in 1 2 0; do
  GG_CG_RQ=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rq$m -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline off --lanczos 0 --grief off > $O/b$m.json 2> $O/b$m.err || { tail -5 $O/b$m.err; exit 1; }
done
for m in 1 2 0; do
  f=$(find $O/rq$m -name "*kernel_stats.csv" | head -1)
  echo "rq=$m"; python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'mode_product' in r['Name'] or 'cg_' in r['Name']:
        print('%8.3f ms x%-4s %s' % (float(r['AverageNs'])/1e6, r['Calls'], r['Name'].split('(')[0][-70:]))
"
done
echo done
