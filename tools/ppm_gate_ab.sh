#!/bin/bash
# Gate-variant A/B on one GPU box: PPM GPU parity of each lib/libceng795_ppm_<v>.so variant,
# then tools/ppm_ab.sh's diag timers and interleaved C5 timings ("new" = production build).
#   tools/ppm_gate_ab.sh <outdir> "<variants>"
set -o pipefail
O=${1:-gpurun_out/ppm_gate}; V=${2:-"new g4"}; mkdir -p $O
for v in $V; do
  [ $v = new ] && continue
  CENG795_PPM_LIB=$v timeout -k 10 400 python -u -m pytest tests/test_ppm_gpu.py -x -q -k "updates or compaction or batched" --timeout 300 --timeout-method thread > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
  echo "$v parity: $(tail -1 $O/tests_$v.log)"
done
bash tools/ppm_ab.sh $O "$V"
