#!/bin/bash
# Round 5: frames in flight per rank of the split (4 / 6 / 8), the N = 1 line's prediction.
set -o pipefail
O=gpurun_out/r05x2
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do for f in 2 3 4; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --split-inflight $f --no-c5 --no-cpu-baseline \
    --no-roofline > $O/f${f}_$r.json 2> $O/f${f}_$r.err || { tail -20 $O/f${f}_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/f${f}_$r.json').read().strip().splitlines()[-1])
p=d['predicted_strong_scaling']; c=d['predicted_strong_scaling_c4']
print('f$f r$r', d['value'], p['t1_ms'], 'c3', {n: (max(v['bands_records']['band_ms_per_rank']), v['predicted_efficiency'], v['bands']['predicted_efficiency']) for n,v in p['per_n'].items()}, 'c4', {n: (v['predicted_efficiency'], v['bands']['predicted_efficiency']) for n,v in c['per_n'].items()})"
done; done
