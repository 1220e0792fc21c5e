#!/bin/bash
# Round 5: HW queues x frames in flight, with the share probe on the bench's own streams.
set -o pipefail
O=gpurun_out/r05s
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do for v in "4 4" "8 4" "8 6" "4 6"; do set -- $v
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --inflight $2 --no-c5 \
    --no-cpu-baseline --no-roofline > $O/q$1_f$2_$r.json 2> $O/q$1_f$2_$r.err || { tail -20 $O/q$1_f$2_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/q$1_f$2_$r.json').read().strip().splitlines()[-1])
p=d['predicted_strong_scaling']; c=d['predicted_strong_scaling_c4']
print('q$1 f$2 r$r', d['value'], p['t1_ms'], 'c3 n8', p['per_n']['8']['bands']['band_ms_max'], max(p['per_n']['8']['bands_records']['band_ms_per_rank']), 'n4', p['per_n']['4']['bands']['band_ms_max'], 'c4', c['t1_ms'], c['per_n']['8']['bands']['band_ms_max'], max(c['per_n']['8']['bands_records']['band_ms_per_rank']))"
done; done
