#!/bin/bash
# Round 5: C5 photon kernel occupancy (waves per EU 6 / 7 vs the shipped build), interleaved.
set -o pipefail
O=gpurun_out/r05y
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do for v in base pw6 pw7; do
  if [ $v = base ]; then L=""; else L=$v; fi
  CENG795_PPM_LIB=$L timeout -k 10 240 python3 -u bench.py --workload c5 --steps 10 --warmup 2 \
    --no-cpu-baseline > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -20 $O/${v}_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1])
print('$v r$r', d['value'], d['ms_per_step'], d['roofline'].get('achieved'))"
done; done
