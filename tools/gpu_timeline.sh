#!/bin/bash
# Wave timelines (RT_TIMELINE build) of the traversal kernels for dispatch-order settings.
set -o pipefail
O=gpurun_out/${1:-timeline}; mkdir -p $O
export TMPDIR=/tmp
for cfg in "2 1" "2 0" "0 0"; do
  set -- $cfg
  CENG795_LIB=timeline CENG795_RT_ORDER=$1 CENG795_RT_PROBE=$2 timeout -k 10 120 python3 tools/timeline.py --slots 7168 --save $O/maps_o$1p$2.npz > $O/tl_o$1p$2.json 2> $O/tl.err || { tail -20 $O/tl.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/tl_o$1p$2.json'))
for k,v in d.items(): print('o$1p$2', k[:20], v['span_us'], v['last_start_us'], v['wave_us_p10_p50_p90_max'], v['slot_utilisation'])"
done
