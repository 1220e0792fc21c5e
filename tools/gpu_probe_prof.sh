#!/bin/bash
# Kernel-level breakdown of the probe-ordered primary pass (rocprofv3 kernel stats).
set -o pipefail
O=gpurun_out/${1:-probe_prof}; mkdir -p $O
export TMPDIR=/tmp
for cfg in "2 1" "2 0"; do
  set -- $cfg
  CENG795_RT_ORDER=$1 CENG795_RT_PROBE=$2 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/o$1p$2 -o run --output-format csv -- python3 tools/kt.py --frames 20 > $O/o$1p$2.out 2>&1 || { tail -20 $O/o$1p$2.out; exit 1; }
  echo "o$1p$2"; python3 tools/trace_iso.py $O/o$1p$2/run_kernel_trace.csv
done
for rep in 1 2; do
  for cfg in "2 0" "2 1"; do
    set -- $cfg
    CENG795_RT_ORDER=$1 CENG795_RT_PROBE=$2 timeout -k 10 120 python3 tools/kt.py >> $O/kt.jsonl 2>> $O/kt.err || { tail -20 $O/kt.err; exit 1; }
    tail -1 $O/kt.jsonl
  done
done
