#!/bin/bash
# Shadow-kernel HBM traffic vs dispatch order (verdict r02 item 5): FETCH_SIZE / WRITE_SIZE /
# TCC passes of one-frame-at-a-time C3 renders for CENG795_RT_ORDER = 0, 1, 2.
set -o pipefail
O=gpurun_out/${1:-shadow_traffic}; mkdir -p $O
export TMPDIR=/tmp
for o in 0 1 2; do
  CENG795_RT_ORDER=$o bash tools/pmc_passes.sh $O/o$o traffic || exit 1
  python3 tools/pmc_traffic.py --fetch $O/o$o/fetch --write $O/o$o/write --out $O/traffic_o$o.json > $O/o$o.sum 2>&1 || { cat $O/o$o.sum; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/traffic_o$o.json'))
for k,v in d['per_kernel'].items(): print('order $o', k, v['read_bytes_corrected'], v['write_bytes'], v['dispatches'])"
done
