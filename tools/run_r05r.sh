#!/bin/bash
# Round 5: the bench with 8 HW queues / 6 frames in flight, probe on the bench's own streams (x2);
# two-rank gloo test.
set -o pipefail
O=gpurun_out/r05t
mkdir -p $O
export TMPDIR=/tmp
for k in 1 2; do
  timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > $O/bench$k.json 2> $O/bench$k.err || { tail -20 $O/bench$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench$k.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['one_frame_ms'], d['cold_frame_ms'], d['roofline']['frac'], d['c5']['value'])
for key in ['predicted_strong_scaling','predicted_strong_scaling_c4']:
  p=d[key]; print(key, p['t1_ms'], {n:(v['predicted_efficiency'], v['bands']['predicted_efficiency'], v['bands_records']['band_ms_per_rank'], v['render_stream_sets_ms']) for n,v in p['per_n'].items()})"
done
timeout -k 10 600 python3 -u -m pytest tests/test_full_configs_gpu.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "two_ranks or rehearsal" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
