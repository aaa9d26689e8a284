#!/bin/bash
# round 3: P2 tests after the WEB CholeskyQR3 SVD, LML factor reuse, ticketed chains
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r03l
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_web.py tests/test_gpu_grief.py tests/test_gpu_configs.py tests/test_gpu_grief_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -30; exit $rc; }

timeout -k 10 300 python -u -m pytest tests/test_gpu_kron.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_kron.log 2>&1; rc=$?
tail -1 $O/pytest_kron.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest_kron.log | head -30; exit $rc; }
timeout -k 10 300 python -u tools/shard_compute.py > $O/shard_compute.jsonl 2> $O/shard.err || { tail -5 $O/shard.err; exit 1; }
cat $O/shard_compute.jsonl
echo done
