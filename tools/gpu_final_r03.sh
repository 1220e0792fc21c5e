#!/bin/bash
# Round-3 closing run on one GPU box: the full checkpoint (tools/gpu_full_r03.sh: GPU suite,
# smoke, default bench line, one-frame-at-a-time kernel stats, RCCL rehearsal, C3 PMC passes)
# plus the C5 PMC traffic passes of the shipping PPM library and a C5 kernel-stats profile;
# then the default bench line again, now with both traffic files matching the libraries.
#   tools/gpu_final_r03.sh <name>
set -o pipefail
N=${1:-final}; O=gpurun_out/$N
export TMPDIR=/tmp
bash tools/gpu_full_r03.sh $N pmc || exit 1
BENCH_ARGS="--workload c5" bash tools/pmc_passes.sh $O/pmc5 traffic || exit 1
python3 tools/pmc_traffic.py --fetch $O/pmc5/fetch --write $O/pmc5/write --workload c5 --round r03 \
  --lib ceng795_amd/lib/libceng795_ppm.so --out $O/traffic_c5.json > /dev/null || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof5 -o run --output-format csv -- python3 bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline > $O/prof5.out 2>&1 || { tail -20 $O/prof5.out; exit 1; }
cp $O/traffic_c3.json profiles/traffic_c3.json && cp $O/traffic_c5.json profiles/traffic_c5.json
timeout -k 10 600 python3 -u bench.py > $O/bench_final.json 2> $O/bench_final.err || { tail -20 $O/bench_final.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_final.json').read().strip().splitlines()[-1])
r=d['roofline']; c=d.get('c5') or {}; cr=c.get('roofline') or {}
print('final c3', d['value'], d['ms_per_step'], 'frac', r['frac'], 'traffic', r['traffic'])
print('final c5', c.get('value'), c.get('ms_per_step'), 'update', cr.get('kernel_ms_avg'), 'frac', cr.get('frac'), 'traffic', cr.get('traffic'))"
