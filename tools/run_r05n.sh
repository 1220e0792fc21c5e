#!/bin/bash
# Round 5: the row-band split (tile costs, band parity, rehearsals) and the bench with its
# band / tile predictions.
set -o pipefail
O=gpurun_out/r05n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bands.py tests/test_gpu_records.py tests/test_gpu_parity.py tests/test_gpu_multi.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $O/bands.log 2>&1 || { tail -30 $O/bands.log; exit 1; }
tail -1 $O/bands.log
timeout -k 10 600 python3 -u -m pytest tests/test_full_configs_gpu.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -k "rehearsal" > $O/rehearsal.log 2>&1 || { tail -20 $O/rehearsal.log; exit 1; }
tail -1 $O/rehearsal.log
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err \
  || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d.get('one_frame_ms'), d.get('cold_frame_ms'), d['roofline']['kernel_ms_avg'], d['roofline']['frac'])
for key in ['predicted_strong_scaling','predicted_strong_scaling_c4']:
  p=d[key]; print(key, p['t1_ms'])
  for n,v in p['per_n'].items():
    print('  ', n, v['predicted_efficiency'], 'bands', v['bands']['band_ms_max'], v['bands']['predicted_efficiency'], v['bands']['peer_link_MB_per_step_max'], 'rec', v['bands_records']['band_ms_per_rank'], v['bands_records']['predicted_efficiency'], v['bands_records']['peer_link_MB_per_step_max'], v['bands_records']['resolve_frac_of_frame'], 'tiles', v['tiles']['predicted_efficiency'])
print('c5', d['c5']['value'])"
