#!/bin/bash
# Round 5: counters and kernel summaries of the shipping libraries, then a bench line that
# carries them (profiles/traffic_c3.json keyed by the library's sha256).
set -o pipefail
O=gpurun_out/r05f
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu.sh r05f pmc c3 r05 || exit 1
cp $O/traffic_c3.json profiles/traffic_c3.json || exit 1
bash tools/gpu.sh r05f stats c3_inflight1 --steps 20 --warmup 5 --inflight 1 --no-cpu-baseline \
  --no-c5 --no-share-probe || exit 1
bash tools/gpu.sh r05f stats c5 --workload c5 --steps 3 --warmup 1 --no-cpu-baseline || exit 1
bash tools/gpu.sh r05f bench bench_final --steps 20 --warmup 5 || exit 1
echo all done
