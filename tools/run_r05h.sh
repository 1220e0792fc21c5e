#!/bin/bash
# Round 5: the driver's bench command with device preconditioning, twice; rehearsal tests.
set -o pipefail
O=gpurun_out/r05h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_full_configs_gpu.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k rehearsal > $O/rehearsal.log 2>&1 || { tail -20 $O/rehearsal.log; exit 1; }
tail -1 $O/rehearsal.log
for k in 1 2; do
  timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > $O/bench$k.json 2> $O/bench$k.err \
    || { tail -20 $O/bench$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench$k.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['config']['preconditioning'], d.get('one_frame_ms'), d.get('cold_frame_ms'), d['roofline']['kernel_ms_avg'], d['roofline']['frac'], d['roofline']['traffic'])
for key in ['predicted_strong_scaling','predicted_strong_scaling_c4']:
  p=d[key]; print(key, p['t1_ms'], {n:(v['share_ms_max'], v['predicted_efficiency']) for n,v in p['per_n'].items()})
print('c5', d['c5']['value'])"
done
