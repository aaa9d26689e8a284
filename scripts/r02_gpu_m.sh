#!/bin/bash
# Round 2, session m: Cholesky look-ahead on a low-priority stream (check,
# timings, kernel traces with / without look-ahead); Phi writer 64 rows per
# block (tests + GRIEF bench); SQ counters of the fused-CG mode products.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02m
mkdir -p $O
timeout -k 10 300 python -u tools/potrf_check.py 1000,5000,10000 > $O/potrf_check.jsonl 2> $O/potrf_check.err || { tail -5 $O/potrf_check.err; exit 1; }
cat $O/potrf_check.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_grief.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_p2.log 2>&1; rc=$?
tail -2 $O/pytest_p2.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_p2.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/p2_kernels_bench.py --what potrf --shapes 100000x10000 > $O/potrf.jsonl 2> $O/potrf.err || { tail -5 $O/potrf.err; exit 1; }
cat $O/potrf.jsonl
GG_POTRF_LOOKAHEAD=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_potrf_nola -o run -- python -u tools/p2_kernels_bench.py --what potrf --shapes 100000x10000 > $O/potrf_nola.jsonl 2> $O/potrf_nola.err || { tail -5 $O/potrf_nola.err; exit 1; }
cat $O/potrf_nola.jsonl
timeout -k 10 600 python -u bench_grief.py --configs C2,C5 --repeats 2 --cpu off > $O/bench_grief.jsonl 2> $O/bench_grief.err || { tail -5 $O/bench_grief.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r02m/bench_grief.jsonl"):
    d=json.loads(l); print(d["config"]["workload"], round(d["fit_ms"],2), {k: round(v,2) for k,v in d["stage_ms"].items()}, "phi frac", round(d["phi"]["frac"],3))
PY
B="python -u bench.py --steps 2 --warmup 1 --cpu-baseline off"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAIT_INST_LDS --kernel-trace -d $O/mp_sq -o run --output-format csv -- $B > $O/mp_sq.log 2>&1 || { tail -5 $O/mp_sq.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-trace -d $O/mp_sq2 -o run --output-format csv -- $B > $O/mp_sq2.log 2>&1 || { tail -5 $O/mp_sq2.log; exit 1; }
echo done
