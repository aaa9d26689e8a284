#!/bin/bash
# Round 2, session n: Cholesky chain on a high-priority stream (check +
# timing); eigensolver with the hand-unrolled QL chain (tests + phases); GRIEF
# C5 kernel trace (Phi writer time).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02n
mkdir -p $O
timeout -k 10 300 python -u tools/potrf_check.py 1000,5000,10000 > $O/potrf_check.jsonl 2> $O/potrf_check.err || { tail -5 $O/potrf_check.err; exit 1; }
cat $O/potrf_check.jsonl
timeout -k 10 300 python -u tools/p2_kernels_bench.py --what potrf --shapes 100000x5000,100000x10000 > $O/potrf.jsonl 2> $O/potrf.err || { tail -5 $O/potrf.err; exit 1; }
cat $O/potrf.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_kron.py tests/test_gpu_grief.py -m gpu -x -q --timeout 120 --timeout-method thread -k "eigensolver or schur or grid_gp or fixture or automobile or fd_gradient or cholesky" > $O/pytest_eig.log 2>&1 || { tail -30 $O/pytest_eig.log; exit 1; }
echo "eig tests: $(tail -1 $O/pytest_eig.log)"
GG_EIG_PROF=1 timeout -k 10 120 python -u tools/p2_kernels_bench.py --what eig > $O/eig_prof.log 2>&1 || { tail -5 $O/eig_prof.log; exit 1; }
grep -E "\"eig\"" $O/eig_prof.log; grep "eig m=" $O/eig_prof.log | awk '!seen[$2]++'
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_grief -o run -- python -u bench_grief.py --configs C5 --repeats 1 --cpu off > $O/bench_grief.jsonl 2> $O/bench_grief.err || { tail -5 $O/bench_grief.err; exit 1; }
python - <<'PY'
import csv
for r in list(csv.DictReader(open("gpurun_out/r02n/prof_grief/run_kernel_stats.csv")))[:14]:
    print(f'{r["Name"][:70]:70s} calls={r["Calls"]:>6s} total_ms={float(r["TotalDurationNs"])/1e6:9.2f} avg_us={float(r["AverageNs"])/1e3:9.1f}')
PY
