#!/bin/bash
# Ring kernel: parity tests, then the 200^4 A/B against the chunked kernel.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r04_b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/ring_ab.py > $O/ring_ab.jsonl 2> $O/ring_ab.err || { tail -5 $O/ring_ab.err; exit 1; }
cat $O/ring_ab.jsonl
