#!/bin/bash
# GPU test suite, C3 bench (default = 2 frames in flight, and 1), C4, and the 2-rank gloo
# rehearsal of the whole-frame gather on one GPU.
set -o pipefail
O=gpurun_out/${1:-r02x}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.out 2>&1 || { tail -40 $O/gpu_tests.out; exit 1; }
tail -1 $O/gpu_tests.out
timeout -k 10 400 python3 -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
cat $O/bench_c3.json
timeout -k 10 200 python3 -u bench.py --inflight 1 --no-cpu-baseline --no-roofline > $O/bench_c3_inflight1.json 2>/dev/null || exit 1
timeout -k 10 200 python3 -u bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline --no-roofline > $O/bench_c4.json 2>/dev/null || exit 1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo --no-cpu-baseline --no-roofline > $O/bench_gloo2.json 2> $O/bench_gloo2.err || { tail -20 $O/bench_gloo2.err; exit 1; }
for f in bench_c3_inflight1 bench_c4 bench_gloo2; do python3 -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'], d['config']['parallelism'], d['config'].get('gather_verified'))"; done
