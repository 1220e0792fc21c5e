#!/bin/bash
# C5 timings of the production PPM library under values of one environment knob, interleaved
# on one box, after the PPM GPU suite + the full-size C5 parity tests.
#   tools/ppm_env_ab.sh <outdir> <VAR> "<values>" [reps]
set -o pipefail
O=${1:-gpurun_out/ppm_env}; VAR=${2:?variable}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_ppm_gpu.py tests/test_full_configs_gpu.py -k "ppm or c5 or C5 or update or multi or shard or batch" -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in $(seq ${4:-2}); do for v in ${3:?values}; do
  env $VAR=$v timeout -k 10 200 python3 -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5_$v.$r.json 2>$O/c5_$v.$r.err || { tail -5 $O/c5_$v.$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c5_$v.$r.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$VAR=$v', d['ms_per_step'], d['value'], 'photon_ms', d['config']['phase_ms']['photon'], 'update/launch', r['kernel_ms_avg'], 'x', r['launches_per_step'], d['config'].get('updates_per_step'))"
done; done
