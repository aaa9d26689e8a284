#!/bin/bash
# Round 2, session zj: TN Gram split over K against slot quantisation
# (GG_GEMM_SPLITK sweep at the C4 / C5 shapes, then the model's own choice).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02zj
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_grief.py tests/test_abi.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or gram or cholesky or fixtures" > $O/pytest.log 2>&1 || { grep -E "^E |FAILED" $O/pytest.log | head -20; tail -3 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for S in 1 2 3 4 6 8; do
  GG_GEMM_SPLITK=$S timeout -k 10 300 python -u tools/p2_kernels_bench.py --what gram --shapes 100000x5000,100000x10000 > $O/gram_s$S.jsonl 2>> $O/gram.err || exit $?
  python -c "import json;[print('S=$S', json.loads(l)['p'], round(json.loads(l)['ms'],2), round(json.loads(l)['tflops'],1)) for l in open('$O/gram_s$S.jsonl')]"
done
timeout -k 10 300 python -u tools/p2_kernels_bench.py --what gram --shapes 100000x1000,100000x5000,100000x10000 > $O/gram_auto.jsonl 2>> $O/gram.err || exit $?
python -c "import json;[print('auto', json.loads(l)['p'], round(json.loads(l)['ms'],2), round(json.loads(l)['tflops'],1)) for l in open('$O/gram_auto.jsonl')]"
timeout -k 10 600 python -u bench_grief.py --configs C2,C4,C5 --cpu off > $O/bench_grief.jsonl 2> $O/bench_grief.err || { tail -5 $O/bench_grief.err; exit 1; }
python -c "
import json
for l in open('$O/bench_grief.jsonl'):
    d=json.loads(l); print(d['config']['workload'], round(d['fit_ms'],2), {k: round(v,2) for k,v in d['stage_ms'].items()})"
