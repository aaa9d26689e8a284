#!/bin/bash
# round 3, first fold run: fold + kron + C3 parity, bench, kernel stats
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_kron.py tests/test_gpu_c3.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 300 python -u bench.py --cpu-baseline off --lanczos 10 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], [round(v,2) for v in d['mode_product_ms_by_position']], d['roofline']['frac'], d.get('lanczos'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -u bench.py --steps 10 --warmup 2 --cpu-baseline off --lanczos 0 > $O/bench_prof.json 2> $O/bench_prof.err || { tail -5 $O/bench_prof.err; exit 1; }
echo done
