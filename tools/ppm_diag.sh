#!/bin/bash
# Per-phase diag counters (CENG795_PPM_DIAG=2) of C5 for lib/libceng795_ppm_<v>.so variants.
#   tools/ppm_diag.sh <outdir> "<variants>"
set -o pipefail
O=${1:-gpurun_out/ppm_diag}; mkdir -p $O
export TMPDIR=/tmp
for v in ${2:-new}; do  # "new": the shipping source built with -DPPM_PHASE_TIMERS=1 (lib variant "timers")
  L=$v; [ $v = new ] && L=
  CENG795_PPM_DIAG=2 CENG795_PPM_LIB=${L:-timers} timeout -k 10 200 python3 -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline > $O/c5d_$v.json 2>$O/c5d_$v.err || { tail -5 $O/c5d_$v.err; exit 1; }
  echo $v; grep "ppm diag" $O/c5d_$v.err | tail -1
done
