#!/bin/bash
# PPM A/B on one GPU box: GPU parity of the production build, per-phase diag timers and
# interleaved C5 timings of lib/libceng795_ppm_<v>.so variants ("new" = the production build).
#   tools/ppm_ab.sh <outdir> [variants, default "old new"]
set -o pipefail
O=${1:-gpurun_out/ppm_ab}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ppm_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in ${2:-old new}; do
  L=$v; [ $v = new ] && L=
  CENG795_PPM_DIAG=2 CENG795_PPM_LIB=$L timeout -k 10 200 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline > $O/c5d_$v.json 2>$O/c5d_$v.err || { tail -5 $O/c5d_$v.err; exit 1; }
  echo $v; grep "ppm diag" $O/c5d_$v.err | tail -1
done
for r in 1 2; do for v in ${2:-old new}; do
  L=$v; [ $v = new ] && L=
  CENG795_PPM_LIB=$L timeout -k 10 200 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5_$v$r.json 2>$O/c5_$v$r.err || { tail -5 $O/c5_$v$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/c5_$v$r.json')); print('$v', d['ms_per_step'], d['value'])"
done; done
