#!/bin/bash
# Round 5, second call: tile-cost maps of the slow packets, order-kernel skip for small launches,
# more hardware queues / frames in flight for the N = 8 shares.
set -o pipefail
O=gpurun_out/r05b
mkdir -p $O
export TMPDIR=/tmp
for W in 1 8; do
  CENG795_LIB=timeline timeout -k 10 120 python3 tools/timeline.py --world $W --save $O/map_w$W.npz \
    > $O/tl_w$W.json 2> $O/tl_w$W.err || { tail -5 $O/tl_w$W.err; exit 1; }
done
timeout -k 10 600 python3 -u tools/scale_probe.py fused,fusedmt --rounds 2 --workloads c3 > $O/scale_mt.json 2> $O/scale_mt.err \
  || { tail -20 $O/scale_mt.err; exit 1; }
tail -4 $O/scale_mt.err
GPU_MAX_HW_QUEUES=8 timeout -k 10 600 python3 -u tools/scale_probe.py fused,fusedmt --rounds 1 --workloads c3 --inflight 8 \
  > $O/scale_hwq8.json 2> $O/scale_hwq8.err || { tail -20 $O/scale_hwq8.err; exit 1; }
tail -2 $O/scale_hwq8.err

timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err \
  || { tail -20 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
echo all done
