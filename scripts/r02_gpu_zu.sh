#!/bin/bash
# Round 2, session zu: kernel trace of the left-looking panel Cholesky at p = 1e4.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02zu
mkdir -p $O
GG_POTRF_MODE=left timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python -u tools/p2_kernels_bench.py --what potrf --shapes 20000x10000 > $O/p2.jsonl 2> $O/p2.err || { tail -5 $O/p2.err; exit 1; }
cat $O/p2.jsonl
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'potrf_ftrsm' in r['Kernel_Name']]
last = idx[-157:]
seg = rows[last[0] - 1:last[-1] + 1]
t0 = int(seg[0]['Start_Timestamp']); t1 = int(seg[-1]['End_Timestamp'])
print('span us', (t1 - t0) / 1e3)
agg = collections.defaultdict(lambda: [0, 0.0])
for r in seg:
    k = r['Kernel_Name'].split('(')[0][:60]
    agg[k][0] += 1; agg[k][1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
for k, (n, us) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print('%-60s %5d %10.1f us  avg %8.1f' % (k, n, us, us / n))
busy = sum((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in seg)
print('sum of kernel time us %.1f, gaps %.1f' % (busy, (t1 - t0) / 1e3 - busy))
d = [(int(rows[i]['End_Timestamp']) - int(rows[i]['Start_Timestamp'])) / 1e3 for i in last]
for pos in range(4):
    v = d[pos::4]
    print('position', pos, 'avg us %.1f' % (sum(v) / len(v)))
PY
