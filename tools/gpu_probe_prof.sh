#!/bin/bash
# Kernel-level breakdown of the probe-ordered primary pass (rocprofv3 kernel stats).
set -o pipefail
O=gpurun_out/${1:-probe_prof}; mkdir -p $O
export TMPDIR=/tmp
for cfg in "2 1" "2 0"; do
  set -- $cfg
  CENG795_RT_ORDER=$1 CENG795_RT_PROBE=$2 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/o$1p$2 -o run --output-format csv -- python3 tools/kt.py --frames 20 > $O/o$1p$2.out 2>&1 || { tail -20 $O/o$1p$2.out; exit 1; }
  python3 - <<PY
import csv
for r in csv.DictReader(open('$O/o$1p$2/run_kernel_stats.csv')):
    print('o$1p$2', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2), round(float(r['MaxNs'])/1e3,2))
PY
done
