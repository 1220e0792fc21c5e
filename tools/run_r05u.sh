#!/bin/bash
# Round 5: HW queues 4 vs 8 with six frames in flight and picked render streams (N = 1 line only).
set -o pipefail
O=gpurun_out/r05u
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-c5 --no-cpu-baseline \
    --no-roofline --no-share-probe > $O/q${q}_$r.json 2> $O/q${q}_$r.err || { tail -20 $O/q${q}_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/q${q}_$r.json').read().strip().splitlines()[-1])
print('q$q r$r', d['value'], d['ms_per_step'], d['config']['render_stream_sets_ms'])"
done; done
