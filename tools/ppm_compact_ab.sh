#!/bin/bash
# Update-pass tile-list compaction A/B on one GPU box (same library, CENG795_PPM_COMPACT sets
# the threshold, 0 = off): PPM GPU parity, per-phase diag timers, interleaved C5 timings, and
# the full-size C5 parity test.
#   tools/ppm_compact_ab.sh <outdir> [thresholds, default "0 65536"]
set -o pipefail
O=${1:-gpurun_out/ppm_compact}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ppm_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in ${2:-0 65536}; do
  CENG795_PPM_DIAG=2 CENG795_PPM_COMPACT=$v timeout -k 10 200 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline > $O/c5d_$v.json 2>$O/c5d_$v.err || { tail -5 $O/c5d_$v.err; exit 1; }
  echo "compact=$v"; grep "ppm diag" $O/c5d_$v.err | tail -1
done
for r in 1 2; do for v in ${2:-0 65536}; do
  CENG795_PPM_COMPACT=$v timeout -k 10 200 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5_$v.$r.json 2>$O/c5_$v.$r.err || { tail -5 $O/c5_$v.$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/c5_$v.$r.json')); print('compact=$v', d['ms_per_step'], d['value'], d['roofline']['kernel_ms_avg'])"
done; done
timeout -k 10 300 python -u -m pytest tests/test_full_configs_gpu.py -x -q -k c5 --timeout 250 --timeout-method thread > $O/full_c5.log 2>&1 || { tail -30 $O/full_c5.log; exit 1; }
tail -1 $O/full_c5.log
