#!/bin/bash
# Round 2, session zp: per-launch kernel trace of gg_potrf at p = 1e4 (block
# chain durations by position in the panel).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02zp
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python -u tools/p2_kernels_bench.py --what potrf --shapes 20000x10000 > $O/p2.jsonl 2> $O/p2.err || { tail -5 $O/p2.err; exit 1; }
cat $O/p2.jsonl
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
# last potrf call: the final 157 potrf_ftrsm launches and everything between
idx = [i for i, r in enumerate(rows) if 'potrf_ftrsm' in r['Kernel_Name']]
last = idx[-157:]
lo, hi = last[0], last[-1]
seg = rows[lo:hi + 1]
t0 = int(seg[0]['Start_Timestamp']); t1 = int(seg[-1]['End_Timestamp'])
print('chain span us', (t1 - t0) / 1e3)
agg = collections.defaultdict(lambda: [0, 0.0])
for r in seg:
    k = r['Kernel_Name'].split('(')[0][:60]
    agg[k][0] += 1; agg[k][1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
for k, (n, us) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print('%-60s %5d %10.1f us  avg %8.1f' % (k, n, us, us / n))
d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in (rows[i] for i in last)]
for pos in range(4):
    v = d[pos::4]
    print('position in panel', pos, 'avg us %.1f' % (sum(v) / len(v)), 'first/last %.1f %.1f' % (v[0], v[-1]))
# gaps between consecutive chain launches (end of block b -> start of block b+1)
gaps = [(int(rows[last[i+1]]['Start_Timestamp']) - int(rows[last[i]]['End_Timestamp'])) / 1e3 for i in range(len(last) - 1)]
print('gap us: within panel avg %.1f, panel boundary avg %.1f' % (
    sum(g for i, g in enumerate(gaps) if (i + 1) % 4) / max(1, sum(1 for i in range(len(gaps)) if (i + 1) % 4)),
    sum(g for i, g in enumerate(gaps) if (i + 1) % 4 == 0) / max(1, sum(1 for i in range(len(gaps)) if (i + 1) % 4 == 0))))
PY
