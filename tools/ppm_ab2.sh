#!/bin/bash
# PPM A/B on one GPU box: GPU parity of the production build (PPM suite + full-size C5 vs the
# golden), then interleaved C5 timings of lib/libceng795_ppm_<v>.so variants ("new" = the
# production build): frame ms, update-kernel ms, Mphotons/s.
#   tools/ppm_ab2.sh <outdir> [variants, default "old new"] [reps, default 2]
set -o pipefail
O=${1:-gpurun_out/ppm_ab}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_ppm_gpu.py tests/test_full_configs_gpu.py -k "ppm or c5 or C5" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in $(seq ${3:-2}); do for v in ${2:-old new}; do
  L=$v; [ $v = new ] && L=
  CENG795_PPM_LIB=$L timeout -k 10 200 python3 -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5_$v$r.json 2>$O/c5_$v$r.err || { tail -5 $O/c5_$v$r.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/c5_$v$r.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['value'], 'update', d['roofline']['kernel_ms_avg'], d['config'].get('updates_per_step'))"
done; done
