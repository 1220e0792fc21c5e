#!/bin/bash
# Probe estimator study: timelines (per-tile primary duration, start, probe estimate) for probe
# depth / visit-cap settings.
set -o pipefail
O=gpurun_out/${1:-probe_est}; mkdir -p $O
export TMPDIR=/tmp
for cfg in "3 48" "5 48" "8 48" "12 64" "40 96"; do
  set -- $cfg
  CENG795_LIB=timeline CENG795_RT_ORDER=2 CENG795_RT_PROBE=1 CENG795_RT_PROBE_DEPTH=$1 CENG795_RT_PROBE_VISITS=$2 timeout -k 10 120 python3 tools/timeline.py --slots 7168 --save $O/maps_d$1v$2.npz > $O/tl_d$1v$2.json 2> $O/tl.err || { tail -20 $O/tl.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/tl_d$1v$2.json'))
for k,v in d.items(): print('d$1v$2', k[:20], v['span_us'], v['last_start_us'], v['wave_us_p10_p50_p90_max'], v['slot_utilisation'])"
done
