#!/bin/bash
# Round 2, session w: left-looking in-panel update inside the Cholesky block
# kernel: check, P2 tests, timings, trace.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02w
mkdir -p $O
timeout -k 10 300 python -u tools/potrf_check.py 300,1000,2500,5000,10000 > $O/potrf_check.jsonl 2> $O/potrf_check.err || { tail -5 $O/potrf_check.err; exit 1; }
cat $O/potrf_check.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_grief.py tests/test_gpu_configs.py tests/test_gpu_web.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_p2.log 2>&1; rc=$?
tail -2 $O/pytest_p2.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_p2.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/p2_kernels_bench.py --what potrf --vendor --shapes 100000x1000,100000x5000,100000x10000 > $O/potrf.jsonl 2> $O/potrf.err || { tail -5 $O/potrf.err; exit 1; }
cat $O/potrf.jsonl
GG_POTRF_LOOKAHEAD=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_potrf_nola -o run -- python -u tools/p2_kernels_bench.py --what potrf --shapes 100000x10000 > $O/potrf_nola.jsonl 2> $O/potrf_nola.err || { tail -5 $O/potrf_nola.err; exit 1; }
cat $O/potrf_nola.jsonl
python - <<'PY'
import csv
for r in list(csv.DictReader(open("gpurun_out/r02w/prof_potrf_nola/run_kernel_stats.csv")))[:6]:
    print(f'{r["Name"][:70]:70s} calls={r["Calls"]:>6s} total_ms={float(r["TotalDurationNs"])/1e6:9.2f} avg_us={float(r["AverageNs"])/1e3:9.1f}')
PY
