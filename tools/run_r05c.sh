#!/bin/bash
# Round 5, third call: the driver's bench command twice with pool-stream renderers.
set -o pipefail
O=gpurun_out/r05c
mkdir -p $O
export TMPDIR=/tmp
for k in 1 2; do
  timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > $O/bench$k.json 2> $O/bench$k.err \
    || { tail -20 $O/bench$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench$k.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d.get('one_frame_ms'), d.get('cold_frame_ms'), d['roofline']['kernel_ms_avg'], d['roofline']['frac'])
for key in ['predicted_strong_scaling','predicted_strong_scaling_c4']:
  p=d[key]; print(key, p['t1_ms'], {n:(v['share_ms_max'], v['predicted_efficiency']) for n,v in p['per_n'].items()})
print('c5', d['c5']['value'])"
done
