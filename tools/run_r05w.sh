#!/bin/bash
# Round 5: frames in flight 5 / 6 / 8 (HIP's 4 hardware queues, picked render streams), N = 1 line.
set -o pipefail
O=gpurun_out/r05w
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do for f in 5 6 8; do
  timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --inflight $f --no-c5 --no-cpu-baseline \
    --no-roofline --no-share-probe > $O/f${f}_$r.json 2> $O/f${f}_$r.err || { tail -20 $O/f${f}_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/f${f}_$r.json').read().strip().splitlines()[-1])
print('f$f r$r', d['value'], d['ms_per_step'], d['config']['render_stream_sets_ms'])"
done; done
