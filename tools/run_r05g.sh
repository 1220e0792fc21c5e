#!/bin/bash
# Round 5: the bench's timed region vs. warm-up length and step count (clock ramp?).
set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
export TMPDIR=/tmp
for a in "20 5" "20 50" "100 5" "20 5" "20 200"; do
  set -- $a
  timeout -k 10 300 python3 -u bench.py --steps $1 --warmup $2 --no-c5 --no-cpu-baseline --no-share-probe \
    --no-roofline > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { tail -5 $O/b_$1_$2.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_$1_$2.json').read().strip().splitlines()[-1])
print('steps $1 warmup $2', d['value'], d['ms_per_step'], d.get('one_frame_ms'))"
done
