#!/bin/bash
# Round 5 closing build (shadow rays enter the first slot): GPU suite, smoke, counters keyed to
# the new library, kernel summaries and the closing bench line.
set -o pipefail
O=gpurun_out/r05z
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu.sh r05z tests || exit 1
cp $O/tests.log $O/gpu_tests.txt
bash tools/gpu.sh r05z smoke || exit 1
bash tools/gpu.sh r05z pmc c3 r05 || exit 1
bash tools/gpu.sh r05z stats c3_final --steps 20 --warmup 5 --no-cpu-baseline --no-c5 \
  --no-share-probe || exit 1
bash tools/gpu.sh r05z stats c3_inflight1 --steps 20 --warmup 5 --inflight 1 --no-cpu-baseline \
  --no-c5 --no-share-probe || exit 1
cp $O/traffic_c3.json profiles/traffic_c3.json || exit 1
bash tools/gpu.sh r05z bench bench_final --steps 20 --warmup 5 || exit 1
echo all done
