#!/bin/bash
# Same-box A/B of the traversal dispatch order: GPU parity first, then
# per-kernel times one frame at a time + 4-in-flight throughput for each order / probe setting,
# interleaved twice.
set -o pipefail
O=gpurun_out/${1:-order_ab}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.out 2>&1 || { tail -40 $O/gpu_tests.out; exit 1; }
tail -1 $O/gpu_tests.out
for rep in 1 2; do
  for cfg in "0 0" "1 0" "2 0" "2 1" "1 1"; do
    set -- $cfg
    CENG795_RT_ORDER=$1 CENG795_RT_PROBE=$2 timeout -k 10 120 python3 tools/kt.py >> $O/kt.jsonl 2>> $O/kt.err || { tail -20 $O/kt.err; exit 1; }
    tail -1 $O/kt.jsonl
  done
done
